#!/bin/bash
# timing A/B builds of attn_fwd_pp64 (tools/v14/pp64.py PP64 knobs):
#   tools/v14/build_pp64_ab.sh NAME [key=val ...] -> tools/diag_libs/libpli_pp64NAME.so
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
N=$1; shift
C=$R/physics-llm-inference_amd/csrc
B=$R/physics-llm-inference_amd/build
python3 $R/tools/v14/pp64.py --ab $N "$@" > /dev/null
mkdir -p $R/tools/diag_libs
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$R/include -I$C \
    "-DPLI_PP64_AB_HEADER=\"$R/tools/ab/pp64_${N}_asm.h\"" -c $C/flash_pp64.hip -o /tmp/ab_pp64$N.o
objs=$(ls $B/*.o | grep -v "/flash_pp64.hip.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs /tmp/ab_pp64$N.o -o $R/tools/diag_libs/libpli_pp64$N.so
echo "built tools/diag_libs/libpli_pp64$N.so ($*)"
