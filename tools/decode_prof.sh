# rocprofv3 kernel trace of graph-replayed decode steps (tools/decode_prof.py)
# for batch ${BATCH:-1}: gpurun_out/dprof_b<B>/, summary via tools/ktrace_layer.py
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
B=${BATCH:-1}
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/dprof_b$B -o dp --output-format csv \
    -- python3 tools/decode_prof.py $B 40 > gpurun_out/dprof_b$B.log 2>&1
