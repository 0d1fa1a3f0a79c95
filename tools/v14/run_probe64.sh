# GPU box: time the head-dim-64 ping-pong probe (prebuilt tools/v14/build/libpp64_probe.so)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/probe64
mkdir -p $O
NAMES=$(grep -o 'X([A-Za-z0-9_]*)' tools/v14/probe64_asm.h | sed 's/X(\(.*\))/\1/' | tr '\n' ' ')
PP_NAMES="$NAMES" NIT=512 ROUNDS=6 timeout -k 10 240 python -u tools/v14/run_probe64.py > $O/probe64.jsonl 2> $O/probe64.err
rc=$?; cat $O/probe64.jsonl; tail -3 $O/probe64.err; exit $rc
