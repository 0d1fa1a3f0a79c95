cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r06_bench}
mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?; python3 -c "import json,sys; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(json.dumps(d['summary']))"; exit $rc
