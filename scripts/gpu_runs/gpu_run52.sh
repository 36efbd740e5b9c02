#!/bin/bash
# Balanced phased chunks and the phased form below 3 chunks, 8 MiB - 512 MiB shards.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r52; mkdir -p $O
timeout -k 10 300 ./build/tune/balance_tune 9 > $O/balance.txt 2> $O/balance.err; rc=$?
echo "rc=$rc"; cat $O/balance.txt; tail -n 3 $O/balance.err; exit $rc
