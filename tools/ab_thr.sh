#!/bin/bash
# fallback-body defer threshold A/B: tools/ab/libpli_mu62.so (v10 / v12 at
# THR 8) vs the product (THR 64 for bf16): v10 at D = 64 (the default route
# there) and v12 (71, explicit) at D = 128, scales 1/sqrt(D) and 0.25
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=gpurun_out/thr; mkdir -p $O
export LIBS="tools/ab/libpli_mu62.so physics-llm-inference_amd/pli_hip/libpli_hip.so"
export ROUNDS=5 ITERS=10
for s in 0 0.25; do
  SHAPE="8,32,4096,64" SCALE=$s VARIANT=-1 timeout -k 10 240 python -u tools/ab_flash.py >> $O/ab.jsonl 2>> $O/ab.err || exit $?
  SCALE=$s VARIANT=71 timeout -k 10 240 python -u tools/ab_flash.py >> $O/ab.jsonl 2>> $O/ab.err || exit $?
  CAUSAL=1 SCALE=$s VARIANT=74 timeout -k 10 240 python -u tools/ab_flash.py >> $O/ab.jsonl 2>> $O/ab.err || exit $?
done
