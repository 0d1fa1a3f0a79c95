# round-6 validation: smoke, the whole GPU suite, bench.py, its rocprofv3
# kernel summary, and the two-rank gloo rehearsal's summary keys (one GPU)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${FINAL_TAG:-r06_final}
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; tail -3 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -4 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?; cut -c1-600 $O/bench.json; [ $rc -eq 0 ] || exit $rc
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --flash-only --steps 20 --warmup 5 > $O/bench_prof.json 2> $O/bench_prof.err)
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
if [ -n "$WITH_GLOO2" ]; then
  PLI_BENCH_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_gloo2.json 2> $O/bench_gloo2.err
  rc=$?; tail -c 1500 $O/bench_gloo2.json; echo; exit $rc
fi
