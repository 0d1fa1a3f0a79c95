cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3p
mkdir -p $O
L=""; for n in cur imm w0 s8 adma; do L="$L tools/ab/libpli_w4$n.so"; done
LIBS="$L" SHAPES="4096x4096x4096,8192x8192x8192" timeout -k 10 400 python -u tools/ab_gemm.py > $O/ab_w4v.log 2>&1; rc=$?; echo rc=$rc
grep -v amdgpu.ids $O/ab_w4v.log | python3 -c "
import sys,json
for l in sys.stdin:
    try: d=json.loads(l)
    except Exception: print(l.strip()); continue
    print(d['shape'][0], d['layout'], d['lib'].split('/')[-1], d['TF/s_median'], d['TF/s_min'], d['bitwise_eq_first'])"
