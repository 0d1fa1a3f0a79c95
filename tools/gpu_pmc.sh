# PMC passes over tools/pmc_kernels.py (one counter group per rocprofv3 run, the
# program directly after --), then tools/pmc_summary.py -> gpurun_out/pmc/traffic.json
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/pmc
mkdir -p $O
for ctr in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE"; do
  tag=$(echo $ctr | cut -d' ' -f1)
  [ "$tag" = SQ_VALU_MFMA_BUSY_CYCLES ] && tag=SQ
  (cd /tmp && timeout -k 10 240 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $O/pmc_$tag -o run -- \
      python3 $GRAFT_REPO_ROOT/tools/pmc_kernels.py > $O/pmc_$tag.log 2>&1)
  rc=$?; echo "pmc $tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_summary.py $O $O/traffic.json > /dev/null && python3 -c "
import json; d=json.load(open('$O/traffic.json'))
for k,v in d.items(): print(k, {x: v.get(x) for x in ('hbm_bytes_per_launch','mfma_busy','clock_GHz','SQ_LDS_BANK_CONFLICT','SQ_INSTS_MFMA')})"
