# in-kernel clock of the 16x16x32 timing build vs the 32x32x16 base (both with the defer-max decision ablated)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3zg
mkdir -p $O
DIAG_LIBS="tools/ab/libpli_diag_sbase.so tools/ab/libpli_diag_m16.so" ROUNDS=3 timeout -k 10 200 python -u tools/v12_clock_ab.py > $O/clock_shape.log 2>&1
rc=$?; echo "clock rc=$rc"; grep -v amdgpu.ids $O/clock_shape.log
exit $rc
