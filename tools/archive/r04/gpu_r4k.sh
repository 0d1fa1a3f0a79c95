# gemm_w5 W5_SPLIT A/B (bitwise + TF/s), NT 8192^3 / tp2 shard / NN 4096^3, default route and persistent
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4k
mkdir -p $O
LIBS="physics-llm-inference_amd/pli_hip/libpli_hip.so tools/ab/libpli_w5split.so" VARIANTS=0,43 LAYOUTS=nt,nn \
  SHAPES=8192x8192x8192,8192x8192x4096,4096x4096x4096 ROUNDS=5 timeout -k 10 400 python -u tools/ab_gemm.py > $O/ab.log 2>&1
rc=$?; grep -v amdgpu.ids $O/ab.log; exit $rc
