# gemm_w4v: ablation (one kind of work removed, timing only) and variant 40 vs the
# default route on the bench / TP-shard / FFN shapes
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3t
mkdir -p $O
fmt() { grep -v amdgpu.ids $1 | python3 -c "
import sys,json
for l in sys.stdin:
    try: d=json.loads(l)
    except Exception: print(l.strip()); continue
    print(d['shape'], d['layout'], d['lib'].split('/')[-1], d['variant'], d['TF/s_median'], d['TF/s_min'], d['bitwise_eq_first'])"; }
L=""; for n in base nodma nord nobar noepi; do L="$L tools/ab/libpli_w4$n.so"; done
LIBS="$L" SHAPES="4096x4096x4096,8192x8192x8192" ROUNDS=5 timeout -k 10 300 python -u tools/ab_gemm.py > $O/ab_abl.log 2>&1
rc=$?; echo "abl rc=$rc"; fmt $O/ab_abl.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="40,0" SHAPES="8192x8192x1024,8192x8192x2048,8192x8192x4096,4096x14336x4096,2048x4096x4096,4096x4096x14336" ROUNDS=5 \
    timeout -k 10 300 python -u tools/ab_gemm.py > $O/ab_shapes.log 2>&1
rc=$?; echo "shapes rc=$rc"; fmt $O/ab_shapes.log
