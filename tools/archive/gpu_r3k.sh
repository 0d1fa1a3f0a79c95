cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
R=$(pwd)
O=gpurun_out/r3k
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread "tests/test_gpu_parity.py::test_row_parallel_fp32_partials_error_by_tp" > $O/pytest.log 2>&1; rc=$?; echo pytest_rc=$rc; tail -3 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
# causal walk A/B: rotation (current) vs pair walks (short-first, long-first)
LIBS="tools/ab/libpli_rot0.so tools/ab/libpli_pair1.so tools/ab/libpli_pair2.so" VARIANTS=74 CAUSAL=1 ROUNDS=8 \
  SHAPE="8,32,4096,128;2,32,8192,128;1,64,16384,128" timeout -k 10 300 python -u tools/ab_flash.py > $O/ab_causal_pair.log 2>&1
rc=$?; echo ab_rc=$rc; cat $O/ab_causal_pair.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
for n in rot0 pair1 pair2; do
  cd /tmp && PLI_HIP_LIB=$R/tools/ab/libpli_$n.so PLI_PMC_CAUSAL=1 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace \
     --output-format csv -d $R/$O/pmc_$n -o run -- python3 $R/tools/flash_pmc.py 74 > $R/$O/pmc_$n.log 2>&1
  rc=$?; echo "pmc $n rc=$rc"; cd $R; [ $rc -eq 0 ] || exit $rc
done
python3 - <<'PY'
import csv,glob
for n in ("rot0","pair1","pair2"):
    for f in glob.glob(f"gpurun_out/r3k/pmc_{n}/**/*counter_collection.csv", recursive=True):
        v=[float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "attn_fwd_v12" in r["Kernel_Name"] and r["Counter_Name"]=="FETCH_SIZE"]
        print(n, "fetch GB per launch (x2 gfx950):", [round(x*1024*2/1e9,3) for x in v])
PY
