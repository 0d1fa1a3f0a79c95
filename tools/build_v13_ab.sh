#!/bin/bash
# timing-only A/B builds of attn_fwd_v13's generated body:
#   tools/build_v13_ab.sh NAME [key=val ...]  ->  tools/ab/libpli_v13NAME.so
# keys: ndef, budget, dma_spacing, dma_cost, abl=dma+exp+check (tools/v13/kernel.py)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
N=$1; shift
python3 $R/tools/gen_flash_v13.py --ab $N "$@" > /dev/null
$R/tools/build_ab.sh v13$N flash_v13.hip "-DPLI_V13_AB_HEADER=\"$R/tools/ab/v13_${N}_asm.h\""
