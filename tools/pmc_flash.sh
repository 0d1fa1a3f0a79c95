cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/fpmc
i=0
for ctr in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" "SQ_VALU_MFMA_COEXEC_CYCLES SQ_CYCLES SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  cd /tmp && timeout -k 10 200 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $R/gpurun_out/fpmc/p$i -o run -- python $R/tools/flash_pmc.py 21 30 31 > $R/gpurun_out/fpmc/p$i.log 2>&1
  rc=$?; echo "pass $i ($ctr) rc=$rc"; cd $R
  [ $rc -eq 0 ] || exit $rc
done
