# QSCALE A/B (+ fma ablation), causal QSCALE, and the clock / per-XCD stamps of the product v13
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4n
mkdir -p $O
LIBS="tools/ab/libpli_v13base.so tools/ab/libpli_v13nochk.so tools/ab/libpli_v13nofma.so tools/ab/libpli_v13qs.so" VARIANTS=80 ROUNDS=8 timeout -k 10 300 python -u tools/ab_flash.py > $O/ab.log 2>&1
rc=$?; grep -v amdgpu.ids $O/ab.log; [ $rc -eq 0 ] || exit $rc
CAUSAL=1 LIBS="tools/ab/libpli_v13base.so tools/ab/libpli_v13qs.so" VARIANTS=83 ROUNDS=6 timeout -k 10 300 python -u tools/ab_flash.py > $O/ab_causal.log 2>&1
rc=$?; grep -v amdgpu.ids $O/ab_causal.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/v13_clock.py > $O/clock.log 2>&1
rc=$?; grep -v amdgpu.ids $O/clock.log; exit $rc
