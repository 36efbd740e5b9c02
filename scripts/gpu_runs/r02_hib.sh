#!/bin/bash
# Round 2: deeper bursts / bigger chunks for the 3-8-bucket sweep.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r02h; mkdir -p $O
timeout -k 10 500 ./build/tune/hib_tune 7 3 > $O/hib_tune.txt 2> $O/hib_tune.err; rc=$?
echo "hib rc=$rc"; cat $O/hib_tune.txt; exit $rc
