# GPU box: fp16 pp64 with the P-bit check in the matrix phase (h_hchk=C) against the product
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/pp64_hchk
mkdir -p $O
LIBS="tools/diag_libs/libpli_pp64base.so tools/diag_libs/libpli_pp64hchk.so" VARIANTS=86 DTYPE=fp16 SHAPE="8,32,4096,64;1,32,32768,64;8,8,2048,64" ROUNDS=8 ITERS=10 \
  timeout -k 10 300 python -u tools/ab_flash.py > $O/ab.jsonl 2> $O/ab.err
rc=$?; python3 -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); print(d['lib'].split('/')[-1], d['shape'], round(d['TF/s_median'],1), round(d['TF/s_min'],1), round(d['TF/s_max'],1), d['bitwise_eq_first'])
"; exit $rc
