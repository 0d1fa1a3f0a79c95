# gemm_w6 (variant 42: VGPR-staged) parity, then A/B vs gemm_w5 (41) and hipBLASLt
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3zd
mkdir -p $O
VARIANT=42 SHAPES="4096x4096x4096" ROUNDS=2 timeout -k 10 200 python -u tools/w4v_check.py > $O/w6_check.log 2>&1
rc=$?; echo "w6 check rc=$rc"; grep -v amdgpu.ids $O/w6_check.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
VARIANTS="42,41" SHAPES="4096x4096x4096,8192x8192x8192,8192x8192x1024,4096x14336x4096" ROUNDS=5 \
    timeout -k 10 300 python -u tools/ab_gemm.py > $O/ab_w6.log 2>&1
rc=$?; echo "ab rc=$rc"; [ $rc -eq 0 ] || exit $rc; grep -v amdgpu.ids $O/ab_w6.log | python3 -c "
import sys,json
for l in sys.stdin:
    try: d=json.loads(l)
    except Exception: print(l.strip()); continue
    print(d['shape'], d['layout'], d['variant'], d['TF/s_median'], d['TF/s_min'], d['bitwise_eq_first'])"
