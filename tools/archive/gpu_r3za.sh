# gemm_w5: RING5 (A / B images on 5 ring positions, DMA split across both halves) vs the two-slot form
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3za
mkdir -p $O
L=""; for n in base r5 d0rd2 r5rd2; do L="$L tools/ab/libpli_w5$n.so"; done
LIBS="$L" VARIANTS=41 SHAPES="4096x4096x4096,8192x8192x8192,8192x8192x1024,4096x14336x4096,264x392x128,1000x776x4096" ROUNDS=5 \
    timeout -k 10 400 python -u tools/ab_gemm.py > $O/ab_w5_r5.log 2>&1
rc=$?; echo "ab rc=$rc"; [ $rc -eq 0 ] || exit $rc
grep -v amdgpu.ids $O/ab_w5_r5.log | python3 -c "
import sys,json
for l in sys.stdin:
    try: d=json.loads(l)
    except Exception: print(l.strip()); continue
    print(d['shape'], d['layout'], d['lib'].split('/')[-1], d['TF/s_median'], d['TF/s_min'], d['bitwise_eq_first'])"
