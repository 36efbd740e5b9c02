#!/bin/bash
# Production phased sum with its launches alternated over two streams (tail overlap).
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r68; mkdir -p $O
timeout -k 10 300 ./build/tune/phase_tune 5 4 > $O/phase.txt 2> $O/phase.err; rc=$?
echo "rc=$rc"; cat $O/phase.txt; tail -n 3 $O/phase.err; exit $rc
