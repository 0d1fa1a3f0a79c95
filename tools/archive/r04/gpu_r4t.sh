# device ramp A/B: fresh bench processes (driver flags --warmup 5 --steps 20), ramp 0 vs 300 ms, alternating
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4t
mkdir -p $O
for i in 1 2 3; do
  for r in ${RAMPS:-0 300}; do
    PLI_BENCH_RAMP_MS=$r timeout -k 10 120 python -u bench.py --flash-only --warmup 5 --steps 20 --no-cpu-baseline > $O/b_${r}_$i.json 2> $O/b_${r}_$i.err
    rc=$?; [ $rc -eq 0 ] || exit $rc
    python3 -c "import json; d=json.load(open('$O/b_${r}_$i.json')); print('ramp $r run $i', round(d['value'],1), round(d['roofline']['kernel_ms'],4))"
  done
done
