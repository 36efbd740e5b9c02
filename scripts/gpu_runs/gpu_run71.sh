#!/bin/bash
# Box-to-box spread of the current build: default bench (headline only) + copy probe, one fresh box per call.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r71_$1; mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-inclusive --no-rowops > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc $(grep -o '"avg_kernel_ms": [0-9.]*' $O/bench.json) $(grep -o '"frac": [0-9.]*' $O/bench.json) $(grep -o '"same_box_copy_GBps": [0-9.]*' $O/bench.json)"; exit $rc
