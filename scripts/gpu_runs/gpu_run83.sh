#!/bin/bash
# Probe: software-pipelined read phase of the phased bucket sum (next stage's loads issued before this stage is consumed) vs production, 8 and 2 buckets, 3 arenas.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r83; mkdir -p $O
timeout -k 10 400 ./build/tune/pipe_tune 7 3 > $O/pipe_a.txt 2> $O/a.err; rc=$?
echo "a rc=$rc"; cat $O/pipe_a.txt; exit $rc
