#!/bin/bash
# Round 2: the production sums over 8 fresh allocations.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r02a; mkdir -p $O
timeout -k 10 400 python -u scripts/tune/sum_alloc.py 8 > $O/sum_alloc2.txt 2> $O/sum_alloc2.err; rc=$?
echo "rc=$rc"; cat $O/sum_alloc2.txt; exit $rc
