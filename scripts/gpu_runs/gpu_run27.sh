#!/bin/bash
# Placement / launch-shape probe of the 8-way sum on one box, twice; counter list.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r27; mkdir -p $O
timeout -k 10 200 ./build/tune/placement_tune 6 > $O/placement_a.txt 2> $O/placement_a.err; rc=$?
echo "a rc=$rc"; cat $O/placement_a.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 ./build/tune/placement_tune 6 > $O/placement_b.txt 2> $O/placement_b.err; rc=$?
echo "b rc=$rc"; cat $O/placement_b.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $GRAFT_REPO_ROOT/$O/counters.txt 2>&1; echo "list rc=$?"
exit 0
