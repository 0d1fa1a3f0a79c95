# gemm_w5 (variant 41: K staged 64 deep, two 64 KiB slots): parity, then A/B vs w4v (40) and the phased tile (0 before round 3 = 13)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3x
mkdir -p $O
VARIANT=41 SHAPES="4096x4096x4096" ROUNDS=2 timeout -k 10 200 python -u tools/w4v_check.py > $O/w5_check.log 2>&1
rc=$?; echo "w5 check rc=$rc"; grep -v amdgpu.ids $O/w5_check.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
VARIANTS="41,40,13" SHAPES="4096x4096x4096,8192x8192x8192,8192x8192x1024,4096x14336x4096" ROUNDS=5 \
    timeout -k 10 300 python -u tools/ab_gemm.py > $O/ab_w5.log 2>&1
rc=$?; echo "ab rc=$rc"; [ $rc -eq 0 ] || exit $rc; grep -v amdgpu.ids $O/ab_w5.log | python3 -c "
import sys,json
for l in sys.stdin:
    try: d=json.loads(l)
    except Exception: print(l.strip()); continue
    print(d['shape'], d['layout'], d['variant'], d['TF/s_median'], d['TF/s_min'], d['bitwise_eq_first'])"
