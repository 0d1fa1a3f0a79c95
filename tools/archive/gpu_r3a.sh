set -o pipefail
mkdir -p gpurun_out/r3a
timeout -k 10 300 python -u tools/ab_flash.py > gpurun_out/r3a/ab.log 2>&1; echo ab_rc=$?; grep lib gpurun_out/r3a/ab.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_flash_v12.py "tests/test_gpu_parity.py::test_calibration_probes" "tests/test_gpu_parity.py::test_flash_stress" "tests/test_gpu_parity.py::test_flash_v12_persistent_seams" > gpurun_out/r3a/pytest.log 2>&1; echo pytest_rc=$?; tail -4 gpurun_out/r3a/pytest.log
timeout -k 10 400 python bench.py > gpurun_out/r3a/bench.json 2> gpurun_out/r3a/bench.err; echo bench_rc=$?; tail -2 gpurun_out/r3a/bench.err
timeout -k 10 200 python tools/v12_clock.py > gpurun_out/r3a/clock.log 2>&1; echo clock_rc=$?; tail -4 gpurun_out/r3a/clock.log
