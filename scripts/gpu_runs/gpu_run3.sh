#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 ./scripts/tune/bucket_tune $((1<<20)) 1024 8 7 > gpurun_out/tune7.txt 2> gpurun_out/tune7.err; rc=$?
echo "tune rc=$rc"; cat gpurun_out/tune7.txt; exit $rc
