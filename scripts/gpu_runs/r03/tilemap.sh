#!/bin/bash
# Round 3 probe 8: tile maps of the wave-map kernel (planned init / gather).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03map}; mkdir -p $O
timeout -k 10 300 ./build/probe/r3_tilemap_tune 7 > $O/r3_tilemap_tune.txt 2> $O/r3_tilemap_tune.err; rc=$?
echo "probe rc=$rc"; cat $O/r3_tilemap_tune.txt; tail -5 $O/r3_tilemap_tune.err; exit $rc
