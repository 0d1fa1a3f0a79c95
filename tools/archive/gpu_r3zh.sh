# PMC HBM traffic of gemm_w5 (4096^3 NN / NT, 8192^3 NT), FETCH_SIZE and WRITE_SIZE in separate passes
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
R=$(pwd)
O=gpurun_out/r3zh
mkdir -p $O
for ctr in FETCH_SIZE WRITE_SIZE; do
  cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $R/$O/pmc_$ctr -o run -- \
      python3 $R/tools/gemm_pmc_probe.py > $R/$O/pmc_$ctr.log 2>&1
  rc=$?; echo "pmc $ctr rc=$rc"; cd $R; [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_summary.py $O $O/traffic_gemm.json > /dev/null; python3 -c "
import json; d=json.load(open('$O/traffic_gemm.json'))
for k,v in d.items(): print(k, {g: round(x['hbm_bytes_per_launch']/1e6,1) for g,x in v['by_grid'].items()})"
