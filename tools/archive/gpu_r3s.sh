# round 3 re-entry: flash MFMA-shape timing ablation (16x16x32 vs 32x32x16, settle
# ablated in both), GPU suite on the restored tree, gemm_w4v vs the default route and hipBLASLt
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3s
mkdir -p $O
LIBS="tools/ab/libpli_sbase.so tools/ab/libpli_sm16.so" ROUNDS=8 timeout -k 10 200 python -u tools/ab_flash.py > $O/ab_m16.log 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids $O/ab_m16.log | tail -4
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread -rf \
    > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 $O/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
SHAPES="4096x4096x4096,8192x8192x8192" ROUNDS=5 timeout -k 10 200 python -u tools/w4v_check.py > $O/w4v_check.log 2>&1
rc=$?; echo "w4v rc=$rc"; grep -v amdgpu.ids $O/w4v_check.log | tail -4
