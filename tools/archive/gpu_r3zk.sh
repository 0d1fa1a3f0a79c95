# gemm_w5 persistent (variant 43): parity, then A/B vs the one-tile-per-workgroup form (41) and hipBLASLt
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3zk
mkdir -p $O
VARIANT=43 SHAPES="4096x4096x4096" ROUNDS=2 timeout -k 10 200 python -u tools/w4v_check.py > $O/w5p_check.log 2>&1
rc=$?; echo "w5p check rc=$rc"; grep -v amdgpu.ids $O/w5p_check.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
VARIANTS="43,41" SHAPES="8192x8192x1024,8192x8192x2048,8192x8192x8192,4096x14336x4096,4096x4096x4096,16384x8192x1024" ROUNDS=5 \
    timeout -k 10 300 python -u tools/ab_gemm.py > $O/ab_w5p.log 2>&1
rc=$?; echo "ab rc=$rc"; [ $rc -eq 0 ] || exit $rc; grep -v amdgpu.ids $O/ab_w5p.log | python3 -c "
import sys,json
for l in sys.stdin:
    try: d=json.loads(l)
    except Exception: print(l.strip()); continue
    print(d['shape'], d['layout'], d['variant'], d['TF/s_median'], d['TF/s_min'], d['bitwise_eq_first'])"
