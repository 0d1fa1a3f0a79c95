# gemm_w5 ablations (timing only): no DMA / no fragment reads / no barriers / MFMAs only
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4p
mkdir -p $O
LIBS="tools/ab/libpli_w5base.so tools/ab/libpli_w5nodma.so tools/ab/libpli_w5nord.so tools/ab/libpli_w5nobar.so tools/ab/libpli_w5mfma.so" VARIANTS=0 LAYOUTS=nt,nn \
  SHAPES=8192x8192x8192,8192x8192x4096 ROUNDS=5 timeout -k 10 400 python -u tools/ab_gemm.py > $O/ab.log 2>&1
rc=$?; grep -v amdgpu.ids $O/ab.log | cut -c1-220; exit $rc
