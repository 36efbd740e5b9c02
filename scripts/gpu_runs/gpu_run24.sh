#!/bin/bash
# Row-op kernel forms A/B: per-lane index loads (prod) vs LDS-staged map vs wave __shfl map.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r24
timeout -k 10 300 ./build/tune/rowmap_tune 7 > gpurun_out/r24/rowmap_tune.txt 2> gpurun_out/r24/rowmap_tune.err; rc=$?
echo "rc=$rc"; cat gpurun_out/r24/rowmap_tune.txt; exit $rc
