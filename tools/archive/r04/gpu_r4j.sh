# PMC of TP=1 8192^3 NT: gemm_w5 vs hipBLASLt (traffic, MFMA busy, clock)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r4j
mkdir -p $O
for ctr in FETCH_SIZE "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE"; do
  tag=$(echo $ctr | cut -d' ' -f1); [ "$tag" = SQ_VALU_MFMA_BUSY_CYCLES ] && tag=SQ
  (cd /tmp && PMC_SET=gemm8k timeout -k 10 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $O/pmc_$tag -o run -- \
      python3 $GRAFT_REPO_ROOT/tools/pmc_kernels.py > $O/pmc_$tag.log 2>&1)
  rc=$?; echo "pmc $tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_summary.py $O $O/traffic.json > /dev/null && python3 -c "
import json; d=json.load(open('$O/traffic.json'))
for k,v in d.items(): print(k, {x: v.get(x) for x in ('grid_size','hbm_bytes_per_launch','mfma_busy','clock_GHz','duration_ns_pmc','SQ_LDS_BANK_CONFLICT','SQ_INSTS_LDS','SQ_INSTS_VALU','SQ_WAVES')})"
