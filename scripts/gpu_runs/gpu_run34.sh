#!/bin/bash
# Allocation kind vs the 8-way sum's per-allocation spread, twice on one box.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r34; mkdir -p $O
timeout -k 10 240 ./build/tune/alloc_tune 6 > $O/alloc_a.txt 2> $O/alloc_a.err; rc=$?
echo "a rc=$rc"; cat $O/alloc_a.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 ./build/tune/alloc_tune 6 > $O/alloc_b.txt 2> $O/alloc_b.err; rc=$?
echo "b rc=$rc"; cat $O/alloc_b.txt; exit $rc
