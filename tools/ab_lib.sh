#!/bin/bash
# GPU box: interleaved A/B of builds of the library on the flash bench config.
# LIBS: space-separated .so paths (default: tools/ab/libpli_prev.so and the
# package .so), $ROUNDS alternations, $VARIANTS flash variants.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
LIBS=${LIBS:-"tools/ab/libpli_prev.so physics-llm-inference_amd/pli_hip/libpli_hip.so"}
: > gpurun_out/ab_lib.log
for i in $(seq 1 ${ROUNDS:-2}); do
  for lib in $LIBS; do
    echo "== $lib" >> gpurun_out/ab_lib.log
    PLI_HIP_LIB=$PWD/$lib PLI_FLASH_VARIANTS=${VARIANTS:-55,60} PLI_TUNE_ROUNDS=3 timeout -k 10 200 \
      python -u tools/tune.py flash >> gpurun_out/ab_lib.log 2>&1 || exit $?
  done
done
grep -v amdgpu.ids gpurun_out/ab_lib.log
