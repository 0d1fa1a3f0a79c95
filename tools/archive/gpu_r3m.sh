cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3m
mkdir -p $O
LIBS="tools/ab/libpli_cur.so tools/ab/libpli_ostore.so" VARIANTS=71 ROUNDS=8 \
  SHAPE="8,32,4096,128;16,32,2048,128;4,32,8192,128" timeout -k 10 300 python -u tools/ab_flash.py > $O/ab_ostore.log 2>&1
rc=$?; echo ab_rc=$rc; grep -v amdgpu.ids $O/ab_ostore.log; [ $rc -eq 0 ] || exit $rc
LIBS="tools/ab/libpli_cur.so tools/ab/libpli_ostore.so" VARIANTS=74 CAUSAL=1 ROUNDS=8 \
  SHAPE="8,32,4096,128" timeout -k 10 300 python -u tools/ab_flash.py > $O/ab_ostore_causal.log 2>&1
rc=$?; echo ab_rc=$rc; grep -v amdgpu.ids $O/ab_ostore_causal.log
