#!/bin/bash
# Round 2: write-phase store policy of the sweep sums (write-through vs nt).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r02w; mkdir -p $O
timeout -k 10 500 ./build/tune/wpol_tune 5 2 > $O/wpol_tune.txt 2> $O/wpol_tune.err; rc=$?
echo "wpol rc=$rc"; cat $O/wpol_tune.txt; exit $rc
