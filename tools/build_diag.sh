#!/bin/bash
# Diagnostic library (never the product): flash_v7.hip with PLI_FLASH_STAMPS ->
# tools/libpli_diag.so exporting pli_diag_flash_stamps (tools/flash_stamps.py) and
# pli_diag_gemv (tools/diag/gemv_diag.hip, tools/gemv_stamps.py).
set -e
python3 "$(dirname "$0")/gen_flash_v13.py" --stamp ${STAMP_ARGS:-}
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/physics-llm-inference_amd/csrc
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -fno-honor-nans -DPLI_FLASH_STAMPS \
    ${DIAG_FLAGS:-} -I$R/include -I$C -I$R/tools/diag -shared $C/flash_v7.hip $C/flash_v12.hip $C/flash_v13.hip $C/flash_v13_d64.hip $R/tools/diag/gemv_diag.hip $C/capi.cpp \
    -o ${DIAG_OUT:-$R/tools/libpli_diag.so}
echo "built $R/tools/libpli_diag.so"
