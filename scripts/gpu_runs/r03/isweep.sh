#!/bin/bash
# Round 3 probe 5: wave-local indexed sweep for the planned init / gather.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03isw}; mkdir -p $O
timeout -k 10 300 ./build/probe/r3_isweep_tune 7 > $O/r3_isweep_tune.txt 2> $O/r3_isweep_tune.err; rc=$?
echo "probe rc=$rc"; cat $O/r3_isweep_tune.txt; cat $O/r3_isweep_tune.err | tail -5; exit $rc
