set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_flash_v13_d64.py tests/test_gpu_flash_v13_ragged.py tests/test_gpu_flash_v13.py > gpurun_out/r06/pytest_qsplit.log 2>&1
rc=$?; tail -8 gpurun_out/r06/pytest_qsplit.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
tools/r06_ab.sh gpurun_out/r06/ab3.jsonl 'd64bf16|tools/diag_libs/ab_base.so tools/diag_libs/ab_cand2.so tools/diag_libs/ab_split.so|SHAPE=8,32,4096,64;d64bf16c|tools/diag_libs/ab_base.so tools/diag_libs/ab_cand2.so|SHAPE=8,32,4096,64 CAUSAL=1;d64bf16r|tools/diag_libs/ab_base.so tools/diag_libs/ab_cand2.so|SHAPE=8,32,4000,64;d64bf16s1k|tools/diag_libs/ab_base.so tools/diag_libs/ab_cand2.so|SHAPE=32,32,1024,64;mha512|tools/diag_libs/ab_base.so tools/diag_libs/ab_cand2.so|SHAPE=8,8,2048,64'
