#!/bin/bash
# Round 2: one launch per chunk vs a persistent launch with in-kernel alignment.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r02d; mkdir -p $O
timeout -k 10 500 ./build/tune/persist_tune 7 2 > $O/persist_tune.txt 2> $O/persist_tune.err; rc=$?
echo "persist rc=$rc"; cat $O/persist_tune.txt; exit $rc
