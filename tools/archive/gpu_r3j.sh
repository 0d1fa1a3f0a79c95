cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out/r3j
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread "tests/test_gpu_parity.py::test_row_parallel_fp32_partials_error_by_tp" "tests/test_gpu_parity.py::test_gemm_f32out_vs_f64" > gpurun_out/r3j/pytest.log 2>&1; rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/r3j/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
# GEMV kernel-only time: --quick runs flash + the GEMV leg only (the 16384^2 streaming run is variant 13)
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3j/prof_quick -o run -- \
    python3 $R/bench.py --quick --steps 5 --warmup 5 > $R/gpurun_out/r3j/quick.json 2> $R/gpurun_out/r3j/quick.err
rc=$?; echo "rocprof quick rc=$rc"; cd $R; [ $rc -eq 0 ] || exit $rc
grep gemv_vec gpurun_out/r3j/prof_quick/run_kernel_stats.csv | cut -c1-160
# PMC traffic of the flash and GEMV kernels (separate passes)
for ctr in FETCH_SIZE WRITE_SIZE; do
  cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $R/gpurun_out/r3j/pmc_$ctr -o run -- \
      python3 $R/bench.py --quick --with-decode --steps 3 --warmup 1 > $R/gpurun_out/r3j/pmc_$ctr.json 2> $R/gpurun_out/r3j/pmc_$ctr.err
  rc=$?; echo "pmc $ctr rc=$rc"; cd $R; [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_summary.py gpurun_out/r3j gpurun_out/r3j/traffic.json > /dev/null; cat gpurun_out/r3j/traffic.json | head -40
