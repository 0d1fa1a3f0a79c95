# gemm_w5 tuning sweep (DMA placement, M0 form, rasterization group, read stride) + no-DMA ablation
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3z
mkdir -p $O
L=""; for n in base d0s4 d8s3 d16s3 d1s2 imm0 g8 g2 rd2 nodma; do L="$L tools/ab/libpli_w5$n.so"; done
LIBS="$L" VARIANTS=41 SHAPES="4096x4096x4096,8192x8192x8192,8192x8192x1024" ROUNDS=4 \
    timeout -k 10 400 python -u tools/ab_gemm.py > $O/ab_w5_sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; [ $rc -eq 0 ] || exit $rc
grep -v amdgpu.ids $O/ab_w5_sweep.log | python3 -c "
import sys,json
for l in sys.stdin:
    try: d=json.loads(l)
    except Exception: print(l.strip()); continue
    print(d['shape'], d['layout'], d['lib'].split('/')[-1], d['TF/s_median'], d['TF/s_min'], d['bitwise_eq_first'])"
