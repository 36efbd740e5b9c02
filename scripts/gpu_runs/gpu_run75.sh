#!/bin/bash
# Focused A/B incl. the product wave-map gather (C-ABI, R16) and its R8 form.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r75; mkdir -p $O
ROWMAP_FOCUS=1 timeout -k 10 300 ./build/tune/rowmap_tune 9 > $O/rowmap_focus_a.txt 2> $O/a.err; rc=$?
echo "a rc=$rc"; [ $rc -eq 0 ] || exit $rc
ROWMAP_FOCUS=1 timeout -k 10 300 ./build/tune/rowmap_tune 9 > $O/rowmap_focus_b.txt 2> $O/b.err; rc=$?
echo "b rc=$rc"; cat $O/rowmap_focus_a.txt $O/rowmap_focus_b.txt; exit $rc
