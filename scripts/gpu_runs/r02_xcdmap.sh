#!/bin/bash
# Round 2: block -> tile mapping of the sweep sums (XCD-contiguous, block-contiguous).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r02x; mkdir -p $O
timeout -k 10 500 ./build/tune/xcdmap_tune 5 3 > $O/xcdmap_tune.txt 2> $O/xcdmap_tune.err; rc=$?
echo "rc=$rc"; cat $O/xcdmap_tune.txt; exit $rc
