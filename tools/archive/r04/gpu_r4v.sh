# v13: the V half of the DMA in the PV phase (dma_pv), non-causal and causal
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4v
mkdir -p $O
L=""; for n in base pv8 pv4 pv8s12 pv2s18; do L="$L tools/ab/libpli_v13$n.so"; done
LIBS="$L" VARIANTS=80 ROUNDS=8 timeout -k 10 300 python -u tools/ab_flash.py > $O/ab.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
CAUSAL=1 LIBS="$L" VARIANTS=83 ROUNDS=6 timeout -k 10 300 python -u tools/ab_flash.py > $O/ab_causal.log 2>&1
