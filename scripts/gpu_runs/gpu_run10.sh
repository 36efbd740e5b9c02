#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest10.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest10.log
if [ $rc -ne 0 ]; then exit $rc; fi
B=$GRAFT_REPO_ROOT/build/apps/geeps_clock_bench
timeout -k 10 200 $B 0 1 30100 $((1<<23)) 10 2 > gpurun_out/e2e10.json 2> gpurun_out/e2e10.err; rc=$?
echo "e2e rc=$rc"; cat gpurun_out/e2e10.json gpurun_out/e2e10.err; exit $rc
