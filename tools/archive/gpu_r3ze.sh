# multi-rank rehearsal on one GPU: bench.py --gpus 2 self-launches two ranks (gloo, both ranks on device 0)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3ze
mkdir -p $O
PLI_BENCH_BACKEND=gloo timeout -k 10 900 python bench.py --gpus 2 --steps 10 --warmup 10 --no-cpu-baseline \
    > $O/bench_gpus2_gloo.json 2> $O/bench_gpus2_gloo.err
rc=$?; echo "bench --gpus 2 rc=$rc"; tail -5 $O/bench_gpus2_gloo.err
python3 -c "import json;d=json.load(open('$O/bench_gpus2_gloo.json'));print({k:d.get(k) for k in ('value','n_gpus','ranks_seen','backend','scaling')}); print(d.get('tp_gemm',{}).get('allreduce_us'), d.get('tp_gemm',{}).get('world'))"
exit $rc
