# GPU box: the head-dim-64 ping-pong probe beside attn_fwd_v13_d64 on the same box
# (bench shape and a long one where the per-block seam is ~1 %)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/probe64
mkdir -p $O
NAMES=$(grep -o 'X([A-Za-z0-9_]*)' tools/v14/probe64_asm.h | sed 's/X(\(.*\))/\1/' | tr '\n' ' ')
PP_NAMES="$NAMES" NIT=512 ROUNDS=6 timeout -k 10 240 python -u tools/v14/run_probe64.py > $O/probe64_c.jsonl 2> $O/probe64_c.err
rc=$?; cat $O/probe64_c.jsonl; [ $rc -eq 0 ] || exit $rc
for dt in ${V13_DTYPES-}; do
  LIBS=physics-llm-inference_amd/pli_hip/libpli_hip.so SHAPE="8,32,4096,64;1,32,32768,64;8,32,4096,128" DTYPE=$dt ROUNDS=6 ITERS=10 \
    timeout -k 10 240 python -u tools/ab_flash.py > $O/v13_$dt.jsonl 2> $O/v13_$dt.err
  rc=$?; cat $O/v13_$dt.jsonl; [ $rc -eq 0 ] || exit $rc
done
