#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 ./scripts/tune/rowop_tune $((1<<23)) 7 > gpurun_out/rowtune2.txt 2> gpurun_out/rowtune2.err; rc=$?
echo "rowtune rc=$rc"; cat gpurun_out/rowtune2.txt gpurun_out/rowtune2.err; exit $rc
