# gemm_w5 W5_SPLIT: all / most DMA pieces in half 0 (after the gap-24 barrier)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4u
mkdir -p $O
L=""; for k in t0 t1 t2 t3; do L="$L tools/ab/libpli_w5$k.so"; done
LIBS="$L" VARIANTS=0 LAYOUTS=nt,nn SHAPES=8192x8192x8192,8192x8192x4096,4096x4096x4096 ROUNDS=5 timeout -k 10 500 python -u tools/ab_gemm.py > $O/ab.log 2>&1
