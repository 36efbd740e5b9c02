#!/bin/bash
# Focused A/B: production row-op kernel vs the wave-shfl index map (W = 128 / 1024), two processes.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r74; mkdir -p $O
ROWMAP_FOCUS=1 timeout -k 10 300 ./build/tune/rowmap_tune 9 > $O/rowmap_focus_a.txt 2> $O/a.err; rc=$?
echo "a rc=$rc"; [ $rc -eq 0 ] || exit $rc
ROWMAP_FOCUS=1 timeout -k 10 300 ./build/tune/rowmap_tune 9 > $O/rowmap_focus_b.txt 2> $O/b.err; rc=$?
echo "b rc=$rc"; cat $O/rowmap_focus_a.txt $O/rowmap_focus_b.txt; exit $rc
