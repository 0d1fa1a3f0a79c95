# GPU box: the causal pp64 forms -- the pp64 tests (all forms), then causal
# D = 64 against v13c (83) in one process, both dtypes
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${PP_TAG:-pp64_causal}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_flash_pp64.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for dt in bf16 fp16; do
LIBS=physics-llm-inference_amd/pli_hip/libpli_hip.so VARIANTS=83,86 CAUSAL=1 DTYPE=$dt SHAPE="8,32,4096,64;2,32,8192,64;8,8,2048,64;4,32,1024,64" ROUNDS=6 ITERS=10 \
  timeout -k 10 300 python -u tools/ab_flash.py > $O/ab_$dt.jsonl 2> $O/ab_$dt.err
rc=$?; python3 -c "
import json
for l in open('$O/ab_$dt.jsonl'):
    d=json.loads(l); print('$dt causal', d['variant'], d['shape'], round(d['TF/s_median'],1), d['bitwise_eq_first'], d['max_diff_first'])
"; [ $rc -eq 0 ] || exit $rc
done
