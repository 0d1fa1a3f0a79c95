#!/bin/bash
# GPU box: flash parity tests (-k flash) then an interleaved A/B timing of
# the flash variants in $VARIANTS at the bench config.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "flash" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/w4_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/w4_pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
PLI_FLASH_VARIANTS=${VARIANTS:-21,40,41,42} PLI_TUNE_ROUNDS=4 timeout -k 10 300 python -u tools/tune.py flash > gpurun_out/w4_tune.log 2>&1
rc=$?; echo "tune rc=$rc"; cat gpurun_out/w4_tune.log | tail -12
