#!/bin/bash
# GPU box: attn_fwd_v12 (variant 70) bitwise vs 55 + timing (tools/v12_check.py),
# then the stamped diagnostic build's cycle anatomy (tools/v12_stamps.py).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/v12_check.py > gpurun_out/v12_check.log 2>&1
rc=$?; echo "check rc=$rc"; grep -v amdgpu.ids gpurun_out/v12_check.log | tail -12
[ $rc -eq 0 ] || exit $rc
grep -q ALL_OK gpurun_out/v12_check.log || exit 1
timeout -k 10 120 python -u tools/v12_stamps.py > gpurun_out/v12_stamps.log 2>&1
rc=$?; echo "stamps rc=$rc"; grep -v amdgpu.ids gpurun_out/v12_stamps.log
exit $rc
