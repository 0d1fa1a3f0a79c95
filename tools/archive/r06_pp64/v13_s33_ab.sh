# GPU box: v13 with s33 unused in its non-causal bodies (sNXNT <-> sTD) against the product
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/v13_s33
mkdir -p $O
LIBS="physics-llm-inference_amd/pli_hip/libpli_hip.so tools/diag_libs/libpli_v13s33swap.so" VARIANTS=80 SHAPE="8,32,4096,128;8,32,1024,128;8,32,4096,64" ROUNDS=8 ITERS=10 \
  timeout -k 10 300 python -u tools/ab_flash.py > $O/ab.jsonl 2> $O/ab.err
rc=$?; python3 -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); print(d['lib'].split('/')[-1], d['shape'], round(d['TF/s_median'],1), round(d['TF/s_min'],1), round(d['TF/s_max'],1), d['bitwise_eq_first'])
"; exit $rc
