#!/bin/bash
# Round 3 probe 9: identity-index wave kernel vs y's offset from x.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03camp}; mkdir -p $O
timeout -k 10 300 ./build/probe/r3_camp_tune 7 > $O/r3_camp_tune.txt 2> $O/r3_camp_tune.err; rc=$?
echo "probe rc=$rc"; cat $O/r3_camp_tune.txt; tail -5 $O/r3_camp_tune.err; exit $rc
