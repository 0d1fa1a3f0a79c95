#!/bin/bash
# build the ping-pong timing probe (tools/v14/probe.py -> build/libpp_probe.so); fails on any error
set -eo pipefail
cd "$(dirname "$0")"
python3 probe.py > /dev/null
rm -f build/libpp_probe.so
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 -Wno-inline-asm probe.hip -o build/libpp_probe.so
nm -D build/libpp_probe.so | grep -q pp_launch
echo "built build/libpp_probe.so"
