#!/bin/bash
# GPU box: stall / issue counters of gemm_w5 vs hipBLASLt at 8192^3 NT
# (tools/gemm_pmc_cmp.py), one rocprofv3 --pmc pass per counter group
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
R=$(pwd)
O=$R/gpurun_out/gpmc_cmp
mkdir -p $O
i=0
for ctr in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "GRBM_GUI_ACTIVE SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_IFETCH" \
           "GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $O/p$i -o run -- python3 $R/tools/gemm_pmc_cmp.py > $O/p$i.log 2>&1)
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 - <<'PY'
import csv, glob, collections, json
out = collections.defaultdict(lambda: collections.defaultdict(list))
for p in sorted(glob.glob("gpurun_out/gpmc_cmp/p*/**/*counter_collection.csv", recursive=True)):
    rows = collections.defaultdict(lambda: collections.defaultdict(float)); meta = {}
    for r in csv.DictReader(open(p)):
        d = int(r["Dispatch_Id"]); rows[d][r["Counter_Name"]] += float(r["Counter_Value"])
        meta[d] = r["Kernel_Name"][:40]
    for d, cs in rows.items():
        k = meta[d]
        if "gemm" not in k and "Cijk" not in k:
            continue
        for c, v in cs.items():
            out[k][c].append(v)
res = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in out.items()}
json.dump(res, open("gpurun_out/gpmc_cmp/summary.json", "w"), indent=1)
print(json.dumps(res, indent=1))
PY
