#!/bin/bash
# GPU box: tools/v12_check.py against each library in $LIBS (PLI_HIP_LIB)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/v12_bisect.log
for lib in $LIBS; do
  echo "== $lib" | tee -a gpurun_out/v12_bisect.log
  PLI_HIP_LIB=$PWD/$lib V12_TIME=${V12_TIME:-} timeout -k 10 120 python -u tools/v12_check.py > gpurun_out/v12_one.log 2>&1
  rc=$?
  grep -v "amdgpu.ids\|row_mod64" gpurun_out/v12_one.log | cut -c1-150 | tee -a gpurun_out/v12_bisect.log
  [ $rc -eq 0 ] || { echo "rc=$rc"; exit $rc; }
done
