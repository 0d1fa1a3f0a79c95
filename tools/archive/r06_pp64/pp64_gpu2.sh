# GPU box: attn_fwd_pp64 as the D = 64 bf16 default -- its tests, the D = 64 and
# parity suites, then the product route against v13 (variant 80) in one process
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${PP_TAG:-pp64_2}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_flash_pp64.py tests/test_gpu_flash_v13_d64.py tests/test_gpu_parity.py tests/test_gpu_ch01_ch05.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
LIBS=physics-llm-inference_amd/pli_hip/libpli_hip.so VARIANTS=80,86 SHAPE="8,32,4096,64;1,32,32768,64;8,8,2048,64;4,32,1024,64;2,8,512,64" ROUNDS=6 ITERS=10 \
  timeout -k 10 300 python -u tools/ab_flash.py > $O/ab.jsonl 2> $O/ab.err
rc=$?; python3 -c "
import json
for l in open('$O/ab.jsonl'):
    d=json.loads(l); print(d['variant'], d['shape'], round(d['TF/s_median'],1), d['bitwise_eq_first'])
"; exit $rc
