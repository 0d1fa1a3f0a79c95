mkdir -p gpurun_out/r3f
LIBS="physics-llm-inference_amd/pli_hip/libpli_hip.so tools/ab/libpli_u4.so" SHAPE="8,32,4096,128;2,32,8192,128;32,32,2048,128" ROUNDS=8 timeout -k 10 300 python -u tools/ab_flash.py > gpurun_out/r3f/ab.log 2>&1; echo rc=$?; grep lib gpurun_out/r3f/ab.log
