# persistent gemm_w5 at every K: the GEMM GPU tests (+ deep-K persistent / f32out cases) and the full-size rows
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4s
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_gemm_1wave.py tests/test_gpu_fullsize.py tests/test_gpu_swiglu.py tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; exit $rc
