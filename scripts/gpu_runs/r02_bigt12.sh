#!/bin/bash
# Round 2: bigger sweep chunks (112 / 104 MiB, shallower bursts) and a fused
# last pass, against production at 1, 2 and 8 buckets (scripts/tune/big_tune.hip).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r02bigt; mkdir -p $O
timeout -k 10 400 ./build/tune/big_tune 7 3 > $O/big_tune12.txt 2> $O/big_tune12.err; rc=$?
echo "big_tune rc=$rc"; cat $O/big_tune12.txt; exit $rc
