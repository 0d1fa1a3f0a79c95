# GPU box: pp64 with the scaled-score pairs on v_pk_fma_f32 (pkfma) against the product build, both dtypes
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/pp64_pk
mkdir -p $O
for dt in bf16 fp16; do
LIBS="tools/diag_libs/libpli_pp64base.so tools/diag_libs/libpli_pp64pk.so" VARIANTS=86 DTYPE=$dt SHAPE="8,32,4096,64;1,32,32768,64;8,8,2048,64" ROUNDS=8 ITERS=10 \
  timeout -k 10 300 python -u tools/ab_flash.py > $O/ab_$dt.jsonl 2> $O/ab_$dt.err
rc=$?; python3 -c "
import json
for l in open('$O/ab_$dt.jsonl'):
    d=json.loads(l); print('$dt', d['lib'].split('/')[-1], d['shape'], round(d['TF/s_median'],1), round(d['TF/s_min'],1), round(d['TF/s_max'],1), d['bitwise_eq_first'], d['max_diff_first'])
"; [ $rc -eq 0 ] || exit $rc
done
