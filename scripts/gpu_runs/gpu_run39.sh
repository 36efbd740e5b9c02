#!/bin/bash
# Read/write phase separation for the 8-way sum (LDS-held chunk results), 3 arenas.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r39; mkdir -p $O
timeout -k 10 300 ./build/tune/phase_tune 5 5 > $O/phase.txt 2> $O/phase.err; rc=$?
echo "rc=$rc"; cat $O/phase.txt; tail -3 $O/phase.err; exit $rc
