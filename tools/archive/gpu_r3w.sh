# full GPU suite after the gemm_w4v default switch
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3w
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread -rf \
    > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 $O/pytest_gpu.log
