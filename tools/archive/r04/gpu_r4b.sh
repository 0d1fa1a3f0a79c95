# v13 clock / cycles per wave-tile (diag build) after r4a
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 300 python -u tools/v13_clock.py > $O/clock.log 2>&1
rc=$?; grep -v amdgpu.ids $O/clock.log; exit $rc
