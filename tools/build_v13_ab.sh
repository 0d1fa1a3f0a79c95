#!/bin/bash
# timing-only A/B builds of attn_fwd_v13's generated bodies (D 128 and 64):
#   tools/build_v13_ab.sh NAME [key=val ...]  ->  tools/ab/libpli_v13NAME.so
# keys: ndef, budget, dma_spacing, dma_cost, abl=dma+exp+check, ... (tools/v13/kernel.py Gen)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
N=$1; shift
C=$R/physics-llm-inference_amd/csrc
B=$R/physics-llm-inference_amd/build
python3 $R/tools/gen_flash_v13.py --ab $N "$@" > /dev/null
mkdir -p $R/tools/ab
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$R/include -I$C \
    "-DPLI_V13_AB_HEADER=\"$R/tools/ab/v13_${N}_asm.h\"" -c $C/flash_v13.hip -o /tmp/ab_v13$N.o &
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$R/include -I$C \
    "-DPLI_V13D64_AB_HEADER=\"$R/tools/ab/v13_${N}_d64_asm.h\"" -c $C/flash_v13_d64.hip -o /tmp/ab_v13${N}_d64.o &
wait
objs=$(ls $B/*.o | grep -v "/flash_v13.hip.o" | grep -v "/flash_v13_d64.hip.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs /tmp/ab_v13$N.o /tmp/ab_v13${N}_d64.o -o $R/tools/ab/libpli_v13$N.so
echo "built tools/ab/libpli_v13$N.so ($*)"
