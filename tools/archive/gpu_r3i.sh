mkdir -p gpurun_out/r3i
timeout -k 10 300 python -u tools/warm_order.py > gpurun_out/r3i/warm.log 2>&1; echo rc=$?; tail -2 gpurun_out/r3i/warm.log
