# gemm_w4v: DMA cost vs cache lines per piece (16 x 64-B rows vs 8 x 128-B rows, timing only)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3v
mkdir -p $O
LIBS="tools/ab/libpli_w4base.so tools/ab/libpli_w4lines.so" SHAPES="4096x4096x4096,8192x8192x8192" ROUNDS=5 \
    timeout -k 10 300 python -u tools/ab_gemm.py > $O/ab_lines.log 2>&1
rc=$?; echo "lines rc=$rc"; grep -v amdgpu.ids $O/ab_lines.log | cut -c1-220
