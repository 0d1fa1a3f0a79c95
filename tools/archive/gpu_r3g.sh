mkdir -p gpurun_out/r3g
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_flash_v12.py "tests/test_gpu_parity.py::test_flash_variants_vs_oracle" "tests/test_gpu_parity.py::test_flash_stress" "tests/test_gpu_parity.py::test_flash_full_config_causal" > gpurun_out/r3g/pytest.log 2>&1; rc=$?; echo pytest_rc=$rc; tail -5 gpurun_out/r3g/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
CAUSAL=1 VARIANTS="60,73,74" ROUNDS=6 timeout -k 10 300 python -u tools/ab_flash.py > gpurun_out/r3g/ab_causal.log 2>&1; echo ab_rc=$?; grep lib gpurun_out/r3g/ab_causal.log
LIBS="physics-llm-inference_amd/pli_hip/libpli_hip.so tools/ab/libpli_u4.so" SHAPE="8,32,4096,128;2,32,8192,128;32,32,2048,128" ROUNDS=6 timeout -k 10 300 python -u tools/ab_flash.py > gpurun_out/r3g/ab_u4.log 2>&1; echo ab2_rc=$?; grep lib gpurun_out/r3g/ab_u4.log
