#!/bin/bash
# Round 2: sweep read phase for the 0-2-bucket phased sums (zero-input init, 1 and 2 buckets).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r02l; mkdir -p $O
timeout -k 10 500 ./build/tune/lowb_tune 7 3 > $O/lowb_tune.txt 2> $O/lowb_tune.err; rc=$?
echo "lowb rc=$rc"; cat $O/lowb_tune.txt; exit $rc
