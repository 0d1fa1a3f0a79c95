cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3n
mkdir -p $O
timeout -k 10 300 python -u tools/w4v_check.py > $O/w4v_check.log 2>&1; rc=$?; echo rc=$rc; grep -v amdgpu.ids $O/w4v_check.log
