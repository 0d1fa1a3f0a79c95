#!/bin/bash
# A/B builds of the library that differ only in flash_v12.hip's -D switches:
#   tools/build_v12_ab.sh NAME "-DV12_VPRE=0 ..."  ->  tools/ab/libpli_NAME.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/physics-llm-inference_amd/csrc
B=$R/physics-llm-inference_amd/build
mkdir -p $R/tools/ab
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -fno-honor-nans -I$R/include -I$C $2 \
    -c $C/flash_v12.hip -o /tmp/flash_v12_$1.o
objs=$(ls $B/*.o | grep -v flash_v12.hip.o)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs /tmp/flash_v12_$1.o -o $R/tools/ab/libpli_$1.so
echo "built tools/ab/libpli_$1.so ($2)"
