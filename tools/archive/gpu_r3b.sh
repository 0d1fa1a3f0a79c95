mkdir -p gpurun_out/r3b
timeout -k 10 400 python bench.py > gpurun_out/r3b/bench.json 2> gpurun_out/r3b/bench.err; echo bench_rc=$?; tail -3 gpurun_out/r3b/bench.err
timeout -k 10 200 python -u tools/v12_clock.py > gpurun_out/r3b/clock.log 2>&1; echo clock_rc=$?; tail -4 gpurun_out/r3b/clock.log
