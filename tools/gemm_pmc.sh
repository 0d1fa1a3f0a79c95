#!/bin/bash
# GPU box: PMC passes over tools/gemm_pmc_probe.py -> gpurun_out/gpmc/
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out/gpmc
i=0
for ctr in "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  cd /tmp && timeout -k 10 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $R/gpurun_out/gpmc/p$i -o run -- python3 $R/tools/gemm_pmc_probe.py > $R/gpurun_out/gpmc/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; cd $R
  [ $rc -eq 0 ] || exit $rc
done
python3 - <<'PY'
import csv, glob, collections, json
out = collections.defaultdict(lambda: collections.defaultdict(list))
for p in sorted(glob.glob("gpurun_out/gpmc/p*/**/*counter_collection.csv", recursive=True)):
    rows = collections.defaultdict(lambda: collections.defaultdict(float)); meta = {}
    for r in csv.DictReader(open(p)):
        d = int(r["Dispatch_Id"]); rows[d][r["Counter_Name"]] += float(r["Counter_Value"])
        meta[d] = (r["Kernel_Name"][:60], r.get("Grid_Size", r.get("Grid_Size_X", "")))
    for d, cs in rows.items():
        k = meta[d]
        if "gemm" not in k[0]:
            continue
        for c, v in cs.items():
            out[f"{k[0]}|{k[1]}"][c].append(v)
res = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in out.items()}
json.dump(res, open("gpurun_out/gpmc/summary.json", "w"), indent=1)
print(json.dumps(res, indent=1))
PY
