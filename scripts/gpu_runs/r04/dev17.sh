#!/bin/bash
# Round 4: bench.py's libgeeps legs alone, with the read-my-writes and the
# loopback-TCP (other-node path) legs.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04dev17}; mkdir -p $O
timeout -k 10 400 python -c "import json, bench; print(json.dumps(bench.libgeeps_leg(1 << 20, 1024)))" > $O/libgeeps_leg.json 2> $O/libgeeps_leg.err; rc=$?
echo "leg rc=$rc"; tail -c 3000 $O/libgeeps_leg.json; exit $rc
