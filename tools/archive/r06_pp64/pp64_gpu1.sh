cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/pp64_1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_flash_pp64.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -25 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
LIBS=physics-llm-inference_amd/pli_hip/libpli_hip.so VARIANTS=80,86 SHAPE="8,32,4096,64;1,32,32768,64;8,8,2048,64;4,32,1024,64" ROUNDS=6 ITERS=10 \
  timeout -k 10 300 python -u tools/ab_flash.py > $O/ab.jsonl 2> $O/ab.err
rc=$?; cut -c1-330 $O/ab.jsonl; exit $rc
