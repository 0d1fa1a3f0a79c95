#!/bin/bash
# v13 defer-max offset A/B (PLI_V13_MUOFF builds from tools/build_ab.sh muN):
# scales 1/sqrt(128), 0.25, 1.0, plain and causal, explicit variants 80 / 83
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=gpurun_out/muoff; mkdir -p $O
export LIBS="tools/ab/libpli_mu7.so tools/ab/libpli_mu15.so tools/ab/libpli_mu31.so tools/ab/libpli_mu62.so"
export ROUNDS=5 ITERS=10
for c in 0 1; do
  for s in 0 0.25 1.0; do
    v=80; [ $c -eq 1 ] && v=83
    CAUSAL=$c SCALE=$s VARIANT=$v timeout -k 10 240 python -u tools/ab_flash.py >> $O/ab.jsonl 2>> $O/ab.err || exit $?
  done
done
