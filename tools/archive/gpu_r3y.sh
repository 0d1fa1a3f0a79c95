# flash v12 seam ablation: no O stores at block seams / no next-Q reload / neither (timing only)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3y
mkdir -p $O
L=""; for n in base nost noq noqst; do L="$L tools/ab/libpli_v12$n.so"; done
LIBS="$L" ROUNDS=8 timeout -k 10 300 python -u tools/ab_flash.py > $O/ab_seam.log 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids $O/ab_seam.log | cut -c1-160; [ $rc -eq 0 ] || exit $rc
