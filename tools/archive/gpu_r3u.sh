# flash v12: staggered persistent start (block seams apart in time), same-process A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3u
mkdir -p $O
L=""; for n in 0 1024 2048 4096; do L="$L tools/ab/libpli_stg$n.so"; done
LIBS="$L" ROUNDS=8 SHAPE="8,32,4096,128;2,32,8192,128" timeout -k 10 300 python -u tools/ab_flash.py > $O/ab_stagger.log 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids $O/ab_stagger.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
LIBS="$L" ROUNDS=6 CAUSAL=1 timeout -k 10 300 python -u tools/ab_flash.py > $O/ab_stagger_causal.log 2>&1
rc=$?; echo "ab causal rc=$rc"; grep -v amdgpu.ids $O/ab_stagger_causal.log | cut -c1-200
