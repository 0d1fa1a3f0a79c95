# GPU box: same-process A/B of the pp64 knob builds (tools/v14/build_pp64_ab.sh), variant 86
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${PP_TAG:-pp64_ab}
mkdir -p $O
L=""
for n in ${PP_LIBS:-base dmac sp4 sp8 dmacsp8}; do L="$L tools/diag_libs/libpli_pp64$n.so"; done
LIBS="$L" VARIANTS=86 SHAPE="${PP_SHAPE:-8,32,4096,64;1,32,32768,64}" ROUNDS=${ROUNDS:-6} ITERS=10 \
  timeout -k 10 400 python -u tools/ab_flash.py > $O/ab.jsonl 2> $O/ab.err
rc=$?; python3 -c "
import json,sys
for l in open('$O/ab.jsonl'):
    d=json.loads(l); print(d['lib'].split('/')[-1], d['shape'], round(d['TF/s_median'],1), d['bitwise_eq_first'])
"; exit $rc
