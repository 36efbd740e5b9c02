#!/bin/bash
# Gather of short rows (16 / 64 floats): per-group load vs LDS map vs the product wave map; two processes.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r77; mkdir -p $O
ROWMAP_SHORT=1 timeout -k 10 300 ./build/tune/rowmap_tune 7 > $O/short_a.txt 2> $O/a.err; rc=$?
echo "a rc=$rc"; [ $rc -eq 0 ] || exit $rc
ROWMAP_SHORT=1 timeout -k 10 300 ./build/tune/rowmap_tune 7 > $O/short_b.txt 2> $O/b.err; rc=$?
echo "b rc=$rc"; cat $O/short_a.txt $O/short_b.txt; exit $rc
