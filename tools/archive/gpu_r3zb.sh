# flash v12 stamps (diagnostic build): per-segment cycles per wave-tile incl. the block seam
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3zb
mkdir -p $O
timeout -k 10 200 python -u tools/v12_stamps.py > $O/v12_stamps.log 2>&1
rc=$?; echo "stamps rc=$rc"; grep -v amdgpu.ids $O/v12_stamps.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/v12_clock.py > $O/v12_clock.log 2>&1
rc=$?; echo "clock rc=$rc"; grep -v amdgpu.ids $O/v12_clock.log | tail -4
