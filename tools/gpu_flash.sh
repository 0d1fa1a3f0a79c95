#!/bin/bash
# GPU box: flash parity tests, then an interleaved A/B of the flash variants
# in $VARIANTS at the bench config (non-causal, then causal).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py --maxfail=20 -v -k "flash" --timeout 120 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/flash_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/flash_pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
PLI_FLASH_VARIANTS=${VARIANTS:-21,50,51} PLI_TUNE_ROUNDS=${ROUNDS:-5} timeout -k 10 300 \
    python -u tools/tune.py flash ${EXTRA_LEGS} > gpurun_out/flash_tune.log 2>&1
rc2=$?; echo "tune rc=$rc2"; tail -20 gpurun_out/flash_tune.log
exit $((rc + rc2))
