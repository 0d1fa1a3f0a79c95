# flash v12: defer-max compares inside phase P (slot 20 / 24) vs after it
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3zf
mkdir -p $O
L="tools/ab/libpli_v12base.so tools/ab/libpli_v12mid20.so tools/ab/libpli_v12mid24.so"
LIBS="$L" ROUNDS=8 timeout -k 10 300 python -u tools/ab_flash.py > $O/ab_settle_mid.log 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids $O/ab_settle_mid.log | cut -c1-220; [ $rc -eq 0 ] || exit $rc
LIBS="$L" ROUNDS=6 CAUSAL=1 timeout -k 10 300 python -u tools/ab_flash.py > $O/ab_settle_mid_causal.log 2>&1
rc=$?; echo "ab causal rc=$rc"; grep -v amdgpu.ids $O/ab_settle_mid_causal.log | cut -c1-220
