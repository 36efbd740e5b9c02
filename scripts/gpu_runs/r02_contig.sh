#!/bin/bash
# Round 2: default vs physically contiguous allocation of the 8-way sum's
# arena over fresh allocations (scripts/tune/contig_tune.hip).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r02contig; mkdir -p $O
timeout -k 10 400 ./build/tune/contig_tune 8 > $O/contig_tune.txt 2> $O/contig_tune.err; rc=$?
echo "contig_tune rc=$rc"; cat $O/contig_tune.txt; cat $O/contig_tune.err | tail -3; exit $rc
