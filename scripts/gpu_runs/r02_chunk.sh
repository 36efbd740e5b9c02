#!/bin/bash
# Round 2: chunk size of the sweep-form bucket sum (64 MiB prod vs 96 / 128 MiB).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r02c; mkdir -p $O
timeout -k 10 400 ./build/tune/chunk_tune 7 3 > $O/chunk_tune.txt 2> $O/chunk_tune.err; rc=$?
echo "chunk rc=$rc"; cat $O/chunk_tune.txt; exit $rc
