#!/bin/bash
# GPU-box check: parity tests, a bench line, a rocprofv3 kernel-trace summary.
# Stops at the first crash / timeout (exit status other than 0 or 1).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
MODE=${1:-all}
[ "$MODE" = allpmc ] && RUNALL=1
python -c "import torch;print(torch.cuda.get_device_name(0))" > gpurun_out/device.txt 2>&1
if [ "$MODE" = all ] || [ -n "$RUNALL" ] || [ "$MODE" = tests ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 -rf \
      > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
  ok $rc || exit $rc
fi
if [ "$MODE" = all ] || [ -n "$RUNALL" ] || [ "$MODE" = bench ]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
  [ $rc -eq 0 ] || exit $rc
fi
if [ "$MODE" = all ] || [ -n "$RUNALL" ] || [ "$MODE" = prof ]; then
  cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- \
      python "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --steps 10 --warmup 30 \
      > "$GRAFT_REPO_ROOT/gpurun_out/prof_bench.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/prof.err"
  rc=$?; echo "rocprof rc=$rc"; cd "$GRAFT_REPO_ROOT"
  find gpurun_out/prof -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-250 | head -20
  [ $rc -eq 0 ] || exit $rc
  python tools/trace_check.py gpurun_out/prof/run_kernel_trace.csv gpurun_out/prof_bench.json 30 10
  # headline kernel alone: its stats average is the bench's kernel_ms
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$GRAFT_REPO_ROOT/gpurun_out/prof_flash" -o run -- \
      python "$GRAFT_REPO_ROOT/bench.py" --flash-only --steps 20 --warmup 5 \
      > "$GRAFT_REPO_ROOT/gpurun_out/prof_flash_bench.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/prof_flash.err"
  rc=$?; echo "rocprof flash-only rc=$rc"; cd "$GRAFT_REPO_ROOT"
  [ $rc -eq 0 ] || exit $rc
fi
if [ "$MODE" = pmc ] || [ "$MODE" = allpmc ]; then
  # one counter group per pass (TCC FETCH_SIZE and WRITE_SIZE cannot share a pass)
  rocprofv3 -L > gpurun_out/counters_available.txt 2>&1 || true
  for ctr in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES" "SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT"; do
    tag=$(echo $ctr | tr ' ' '_')
    cd /tmp && timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv \
        -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_$tag" -o run -- \
        python "$GRAFT_REPO_ROOT/bench.py" --quick --with-decode --steps 3 --warmup 1 \
        > "$GRAFT_REPO_ROOT/gpurun_out/pmc_$tag.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/pmc_$tag.err"
    rc=$?; echo "pmc $ctr rc=$rc"; cd "$GRAFT_REPO_ROOT"
    [ $rc -eq 0 ] || exit $rc
  done
  python tools/pmc_summary.py gpurun_out gpurun_out/traffic.json > /dev/null && cat gpurun_out/traffic.json
fi
