# causal walks: A/B 83 vs 84 (and v12 74), FETCH_SIZE per walk
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r4g
mkdir -p $O
CAUSAL=1 LIBS=physics-llm-inference_amd/pli_hip/libpli_hip.so VARIANTS=74,83,84 ROUNDS=8 timeout -k 10 300 python -u tools/ab_flash.py > $O/ab_causal.log 2>&1
rc=$?; grep -v amdgpu.ids $O/ab_causal.log; [ $rc -eq 0 ] || exit $rc
for ctr in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && PMC_SET=causal timeout -k 10 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $O/pmc_$ctr -o run -- \
      python3 $GRAFT_REPO_ROOT/tools/pmc_kernels.py > $O/pmc_$ctr.log 2>&1)
  rc=$?; echo "pmc $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_summary.py $O $O/traffic.json > /dev/null && python3 -c "
import json; d=json.load(open('$O/traffic.json'))
for k,v in d.items(): print(k, json.dumps(v.get('by_grid'))[:600])"
