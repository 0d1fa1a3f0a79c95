#!/bin/bash
# build the head-dim-64 ping-pong timing probe (tools/v14/probe64.py -> build/libpp64_probe.so); fails on any error
set -eo pipefail
cd "$(dirname "$0")"
python3 probe64.py > /dev/null
mkdir -p build
rm -f build/libpp64_probe.so
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 -Wno-inline-asm probe64.hip -o build/libpp64_probe.so
nm -D build/libpp64_probe.so | grep -q pp64_launch
echo "built build/libpp64_probe.so"
