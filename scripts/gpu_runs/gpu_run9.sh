#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
B=$GRAFT_REPO_ROOT/build/apps/geeps_clock_bench
timeout -k 10 200 $B 0 1 30100 $((1<<23)) 10 2 > gpurun_out/e2e9.json 2> gpurun_out/e2e9.err; rc=$?
echo "e2e rc=$rc"; cat gpurun_out/e2e9.json gpurun_out/e2e9.err; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof9" -o run -- $B 0 1 30100 $((1<<23)) 10 2 > "$GRAFT_REPO_ROOT/gpurun_out/prof9.log" 2>&1; rc=$?
echo "rocprof rc=$rc"; exit $rc
