# GPU box: the product pp64 against the pre-causal bodies and the non-persistent build, variant 88
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/pp64_regress
mkdir -p $O
for dt in bf16 fp16; do
LIBS="tools/diag_libs/libpli_pp64nonpers.so tools/diag_libs/libpli_pp64old.so physics-llm-inference_amd/pli_hip/libpli_hip.so" VARIANTS=88 DTYPE=$dt SHAPE="8,32,4096,64;1,32,32768,64" ROUNDS=8 ITERS=10 \
  timeout -k 10 300 python -u tools/ab_flash.py > $O/ab_$dt.jsonl 2> $O/ab_$dt.err
rc=$?; python3 -c "
import json
for l in open('$O/ab_$dt.jsonl'):
    d=json.loads(l); print('$dt', d['lib'].split('/')[-1], d['shape'], round(d['TF/s_median'],1), round(d['TF/s_min'],1), round(d['TF/s_max'],1), d['bitwise_eq_first'])
"; [ $rc -eq 0 ] || exit $rc
done
