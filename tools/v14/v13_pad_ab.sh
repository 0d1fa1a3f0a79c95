# GPU box: v13 with 0 / 1 / 3 / 5 / 8 s_nop before the step loop (its code address moved), same process
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/v13_pad
mkdir -p $O
L=""; for n in p0 p1 p3 p5 p8; do L="$L tools/diag_libs/libpli_v13$n.so"; done
for c in 0 1; do
LIBS="$L" VARIANTS=80 CAUSAL=$c SHAPE="8,32,4096,128" ROUNDS=8 ITERS=10 \
  timeout -k 10 300 python -u tools/ab_flash.py > $O/ab_c$c.jsonl 2> $O/ab_c$c.err
rc=$?; python3 -c "
import json
for l in open('$O/ab_c$c.jsonl'):
    d=json.loads(l); print('causal $c', d['lib'].split('/')[-1], d['shape'], round(d['TF/s_median'],1), round(d['TF/s_min'],1), round(d['TF/s_max'],1), d['bitwise_eq_first'])
"; [ $rc -eq 0 ] || exit $rc
done
