mkdir -p gpurun_out/r3h
LIBS="physics-llm-inference_amd/pli_hip/libpli_hip.so" CAUSAL=1 VARIANTS="60,73,74" SHAPE="8,32,4096,128;2,32,8192,128;32,32,2048,128" ROUNDS=6 timeout -k 10 300 python -u tools/ab_flash.py > gpurun_out/r3h/ab_causal.log 2>&1; echo ab_rc=$?; grep lib gpurun_out/r3h/ab_causal.log | cut -c1-220
