#!/bin/bash
# GPU box: D=64 issue-budget sweep (bf16 / fp16, plain / causal) and the fp16 mu-offset sweep (D128)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=$PWD/gpurun_out/sweep; mkdir -p $O
B="tools/v14/build/libpli_r05cur.so tools/v14/build/libpli_v13b12.so tools/v14/build/libpli_v13b16.so tools/v14/build/libpli_v13b24.so"
for dt in bf16 fp16; do
  DTYPE=$dt SHAPE="8,32,4096,64" LIBS="$B" ROUNDS=5 ITERS=20 timeout -k 10 200 python -u tools/ab_flash.py >> $O/d64_budget.log 2>&1 || exit 1
  DTYPE=$dt CAUSAL=1 SHAPE="8,32,4096,64" LIBS="$B" ROUNDS=5 ITERS=20 timeout -k 10 200 python -u tools/ab_flash.py >> $O/d64_budget.log 2>&1 || exit 1
done
DTYPE=bf16 SHAPE="8,32,4096,128" LIBS="$B" ROUNDS=5 ITERS=20 timeout -k 10 200 python -u tools/ab_flash.py >> $O/d64_budget.log 2>&1 || exit 1
M="tools/v14/build/libpli_r05cur.so tools/v14/build/libpli_muf2.so tools/v14/build/libpli_muf8.so"
DTYPE=fp16 LIBS="$M" ROUNDS=5 ITERS=20 timeout -k 10 200 python -u tools/ab_flash.py >> $O/f16_muoff.log 2>&1 || exit 1
DTYPE=fp16 CAUSAL=1 LIBS="$M" ROUNDS=5 ITERS=20 timeout -k 10 200 python -u tools/ab_flash.py >> $O/f16_muoff.log 2>&1 || exit 1
for f in $O/d64_budget.log $O/f16_muoff.log; do grep -v amdgpu.ids $f | python3 -c "
import sys, json
for l in sys.stdin:
    try: d = json.loads(l)
    except Exception: continue
    print(d['lib'].split('/')[-1], d['shape'][3], 'causal' if d['causal'] else 'plain', round(d['TF/s_median'], 1), d['bitwise_eq_first'], round(d['max_diff_first'], 5))"; done
