# GPU box: pp64 bf16 + fp16 -- its tests, the D = 64 / fp16 / parity suites,
# then the product route against v13 (variant 80) in one process, both dtypes
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${PP_TAG:-pp64_check}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_flash_pp64.py tests/test_gpu_flash_v13_d64.py tests/test_gpu_flash_v13_f16.py tests/test_gpu_parity.py tests/test_gpu_ch01_ch05.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for dt in bf16 fp16; do
LIBS=physics-llm-inference_amd/pli_hip/libpli_hip.so VARIANTS=80,88 DTYPE=$dt SHAPE="8,32,4096,64;1,32,32768,64;8,8,2048,64;4,32,1024,64" ROUNDS=6 ITERS=10 \
  timeout -k 10 300 python -u tools/ab_flash.py > $O/ab_$dt.jsonl 2> $O/ab_$dt.err
rc=$?; python3 -c "
import json
for l in open('$O/ab_$dt.jsonl'):
    d=json.loads(l); print('$dt', d['variant'], d['shape'], round(d['TF/s_median'],1), d['bitwise_eq_first'], d['max_diff_first'])
"; [ $rc -eq 0 ] || exit $rc
done
