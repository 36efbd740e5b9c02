#!/bin/bash
# Phased row ops with the index off the critical path (LDS double-buffered endpoints), 160-KiB chunks.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r47; mkdir -p $O
timeout -k 10 300 ./build/tune/rowphase2_tune 7 > $O/rowphase2.txt 2> $O/rowphase2.err; rc=$?
echo "rc=$rc"; cat $O/rowphase2.txt; tail -n 3 $O/rowphase2.err; exit $rc
