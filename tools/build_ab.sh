#!/bin/bash
# A/B builds of the library that differ only in one source's -D switches:
#   tools/build_ab.sh NAME SRC.hip "-DFOO=1 ..."  ->  tools/ab/libpli_NAME.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/physics-llm-inference_amd/csrc
B=$R/physics-llm-inference_amd/build
mkdir -p $R/tools/ab
X=""
case "$2" in flash_v7.hip|flash_v12.hip) X="-fno-honor-nans";; esac
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $X -I$R/include -I$C $3 \
    -c $C/$2 -o /tmp/ab_$1_$2.o
objs=$(ls $B/*.o | grep -v "/$2.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs /tmp/ab_$1_$2.o -o $R/tools/ab/libpli_$1.so
echo "built tools/ab/libpli_$1.so ($2: $3)"
