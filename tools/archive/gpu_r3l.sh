cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3l
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_flash_v12.py > $O/pytest_v12.log 2>&1; rc=$?; echo pytest_rc=$rc; tail -3 $O/pytest_v12.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --quick --steps 10 --warmup 5 > $O/quick.json 2> $O/quick.err; rc=$?; echo bench_rc=$rc
python3 -c "import json;d=json.loads(open('$O/quick.json').read().strip().splitlines()[-1]);print(d['value'], d['flash_causal'])"
