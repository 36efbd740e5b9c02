#!/bin/bash
# Scatter-add / fused init: production per-group kernel vs the wave map (W 128, 64), two processes.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r79; mkdir -p $O
ROWMAP_SCATTER=1 timeout -k 10 300 ./build/tune/rowmap_tune 7 > $O/scatter_a.txt 2> $O/a.err; rc=$?
echo "a rc=$rc"; [ $rc -eq 0 ] || exit $rc
ROWMAP_SCATTER=1 timeout -k 10 300 ./build/tune/rowmap_tune 7 > $O/scatter_b.txt 2> $O/b.err; rc=$?
echo "b rc=$rc"; cat $O/scatter_a.txt $O/scatter_b.txt; exit $rc
