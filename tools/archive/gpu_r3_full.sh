#!/bin/bash
# Round-3 GPU check: full GPU suite, bench line, rocprofv3 stats (bench and
# flash-only), in-kernel clock, flash PMC passes.  Output under gpurun_out/$OUT.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
R=$(pwd)
OUT=${OUT:-r3full}
mkdir -p gpurun_out/$OUT
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread -rf \
      > gpurun_out/$OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/$OUT/pytest_gpu.log
  ok $rc || exit $rc
fi
timeout -k 10 500 python bench.py > gpurun_out/$OUT/bench.json 2> gpurun_out/$OUT/bench.err
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/$OUT/bench.err; [ $rc -eq 0 ] || exit $rc
python -c "import json;d=json.load(open('gpurun_out/$OUT/bench.json'));print('value',d['value'],'frac',d['roofline']['frac'],'kernel_ms',d['roofline']['kernel_ms'])"
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$OUT/prof -o run -- \
    python3 $R/bench.py --no-cpu-baseline --steps 10 --warmup 30 > $R/gpurun_out/$OUT/prof_bench.json 2> $R/gpurun_out/$OUT/prof.err
rc=$?; echo "rocprof rc=$rc"; cd $R; [ $rc -eq 0 ] || exit $rc
python3 tools/trace_check.py gpurun_out/$OUT/prof/run_kernel_trace.csv gpurun_out/$OUT/prof_bench.json 30 10 > gpurun_out/$OUT/trace_check.txt 2>&1; tail -3 gpurun_out/$OUT/trace_check.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$OUT/prof_flash -o run -- \
    python3 $R/bench.py --flash-only --steps 20 --warmup 5 > $R/gpurun_out/$OUT/prof_flash_bench.json 2> $R/gpurun_out/$OUT/prof_flash.err
rc=$?; echo "rocprof flash rc=$rc"; cd $R; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/v12_clock.py > gpurun_out/$OUT/clock.log 2>&1; echo "clock rc=$?"; tail -3 gpurun_out/$OUT/clock.log
