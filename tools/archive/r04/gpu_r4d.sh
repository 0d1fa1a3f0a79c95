# v13 timing-only ablations and schedule knobs (tools/build_v13_ab.sh), one process, interleaved
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${ABOUT:-r4d}
mkdir -p $O
L=""
for n in ${ABLIBS:-base nochk noexp nokr novr nobar nosoft mfma nodmachk nord}; do L="$L tools/ab/libpli_v13$n.so"; done
LIBS="$L" VARIANTS=80 ROUNDS=8 timeout -k 10 400 python -u tools/ab_flash.py > $O/ab.log 2>&1
rc=$?; grep -v amdgpu.ids $O/ab.log; exit $rc
