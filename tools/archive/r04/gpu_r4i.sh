# causal reversed second blocks: GPU tests (causal), A/B vs the forward-only build, traffic
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r4i
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_flash_v13.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k causal > $O/pytest_causal.log 2>&1
rc=$?; tail -4 $O/pytest_causal.log; [ $rc -eq 0 ] || exit $rc
CAUSAL=1 LIBS="physics-llm-inference_amd/pli_hip/libpli_hip.so tools/ab/libpli_v13fwd.so" VARIANTS=83,84 ROUNDS=8 timeout -k 10 300 python -u tools/ab_flash.py > $O/ab_causal.log 2>&1
rc=$?; grep -v amdgpu.ids $O/ab_causal.log; [ $rc -eq 0 ] || exit $rc
CAUSAL=1 SHAPE="2,16,1024,128;1,8,2048,128;2,32,8192,128" LIBS="physics-llm-inference_amd/pli_hip/libpli_hip.so tools/ab/libpli_v13fwd.so" VARIANTS=83 ROUNDS=3 ITERS=5 timeout -k 10 300 python -u tools/ab_flash.py > $O/ab_causal_shapes.log 2>&1
rc=$?; grep -v amdgpu.ids $O/ab_causal_shapes.log; [ $rc -eq 0 ] || exit $rc
for ctr in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && PMC_SET=causal timeout -k 10 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $O/pmc_$ctr -o run -- \
      python3 $GRAFT_REPO_ROOT/tools/pmc_kernels.py > $O/pmc_$ctr.log 2>&1)
  rc=$?; echo "pmc $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_summary.py $O $O/traffic.json > /dev/null && python3 -c "
import json; d=json.load(open('$O/traffic.json'))
for k,v in d.items(): print(k, json.dumps(v.get('by_grid'))[:600])"
