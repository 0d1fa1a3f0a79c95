# gemm_w5 one-tile (41) vs persistent walk (43) at K >= 8192, current product build
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4r
mkdir -p $O
LIBS="physics-llm-inference_amd/pli_hip/libpli_hip.so" VARIANTS=41,43 LAYOUTS=nt,nn SHAPES=8192x8192x8192,4096x4096x8192,8192x8192x16384,4096x14336x8192 ROUNDS=5 timeout -k 10 500 python -u tools/ab_gemm.py > $O/ab.log 2>&1
rc=$?; exit $rc
