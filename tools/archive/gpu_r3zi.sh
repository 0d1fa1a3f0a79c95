# 16x16x32 timing build with fillers between the two MFMAs of each pair (V12_MF16SPLIT) vs the 32x32x16 base
# (defer-max decision ablated in both): wall TF/s (same process) and in-kernel clock
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3zi
mkdir -p $O
LIBS="tools/ab/libpli_sbase.so tools/ab/libpli_m16s.so" ROUNDS=8 timeout -k 10 300 python -u tools/ab_flash.py > $O/ab_m16s.log 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids $O/ab_m16s.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
DIAG_LIBS="tools/ab/libpli_diag_sbase.so tools/ab/libpli_diag_m16s.so" ROUNDS=2 timeout -k 10 200 python -u tools/v12_clock_ab.py > $O/clock_m16s.log 2>&1
rc=$?; echo "clock rc=$rc"; grep -v amdgpu.ids $O/clock_m16s.log
exit $rc
