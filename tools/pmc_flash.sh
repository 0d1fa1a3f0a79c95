#!/bin/bash
# GPU box: rocprofv3 PMC passes (one counter group per run) over the flash
# variants in $VARIANTS (default 21 30 31) at the bench config, then
# tools/flash_pmc_summary.py -> gpurun_out/fpmc/summary.json
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
R=$(pwd)
VARS=${VARIANTS:-21 30 31}
F=${FPMC_DIR:-gpurun_out/fpmc}
mkdir -p $F
i=0
for ctr in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" "SQ_VALU_MFMA_COEXEC_CYCLES SQ_CYCLES SQ_ACTIVE_INST_ANY" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  cd /tmp && timeout -k 10 200 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $R/$F/p$i -o run -- python3 $R/tools/flash_pmc.py $VARS > $R/$F/p$i.log 2>&1
  rc=$?; echo "pass $i ($ctr) rc=$rc"; cd $R
  [ $rc -eq 0 ] || exit $rc
done
python3 tools/flash_pmc_summary.py $F $VARS > $F/summary.json && cat $F/summary.json
