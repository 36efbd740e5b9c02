#!/bin/bash
# Phase separation for 1R1W copy and the row-indexed gather / scatter-add.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r42; mkdir -p $O
timeout -k 10 300 ./build/tune/rowphase_tune 7 > $O/rowphase.txt 2> $O/rowphase.err; rc=$?
echo "rc=$rc"; cat $O/rowphase.txt; tail -3 $O/rowphase.err; exit $rc
