# causal per-wave stop (skip steps) vs the product library: A/B + bitwise, causal 83/84
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4h
mkdir -p $O
CAUSAL=1 LIBS="physics-llm-inference_amd/pli_hip/libpli_hip.so tools/ab/libpli_v13skip.so" VARIANTS=83,84 ROUNDS=8 timeout -k 10 300 python -u tools/ab_flash.py > $O/ab_causal.log 2>&1
rc=$?; grep -v amdgpu.ids $O/ab_causal.log; [ $rc -eq 0 ] || exit $rc
CAUSAL=1 SHAPE="2,16,1024,128;1,8,2048,128" LIBS="physics-llm-inference_amd/pli_hip/libpli_hip.so tools/ab/libpli_v13skip.so" VARIANTS=83 ROUNDS=2 ITERS=3 timeout -k 10 300 python -u tools/ab_flash.py > $O/ab_causal_small.log 2>&1
rc=$?; grep -v amdgpu.ids $O/ab_causal_small.log; exit $rc
