#!/bin/bash
# GPU box: causal pair-walk orders -- interleaved A/B (B8 H32 S4096 and two
# other pair-walk shapes) and one FETCH_SIZE / WRITE_SIZE pass per library
# (rocprofv3 --pmc, tools/flash_pmc.py variant 83)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=$PWD/gpurun_out/causal_walk
mkdir -p $O
LIBS="${LIBS:-tools/v14/build/libpli_r05cur.so tools/v14/build/libpli_v13sf.so tools/v14/build/libpli_v13fwd.so}"
CAUSAL=1 LIBS="$LIBS" ROUNDS=6 ITERS=20 SHAPE="8,32,4096,128;2,32,8192,128;2,16,1024,128" timeout -k 10 300 python -u tools/ab_flash.py > $O/ab.log 2>&1 || exit $?
for lib in $LIBS; do
  n=$(basename $lib .so)
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && PLI_HIP_LIB=$GRAFT_REPO_ROOT/$lib PLI_PMC_CAUSAL=1 timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_${n}/pmc_$c -o run -- python3 $GRAFT_REPO_ROOT/tools/flash_pmc.py 83 > /dev/null 2>&1) || { echo "pmc $n $c failed"; exit 1; }
  done
  python3 tools/pmc_summary.py $O/pmc_${n} $O/traffic_${n}.json > /dev/null 2>&1 || echo "summary $n failed"
done
grep -v amdgpu.ids $O/ab.log | cut -c1-200
for f in $O/traffic_*.json; do echo $f; python3 -c "import json,sys;d=json.load(open('$f'));k=d.get('attn_fwd_v13c',{});print(k.get('hbm_bytes_per_launch'),k.get('read_bytes_per_launch'))"; done
