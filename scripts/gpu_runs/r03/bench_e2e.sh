#!/bin/bash
# Round 3: the bench's libgeeps clock leg alone (headline step kept short).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03be2e}; mkdir -p $O
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-rowops --no-cpu-baseline --no-host-inclusive --no-config2 --no-per-rank --no-pmc --no-separate-alloc > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; python -c "import json; print(json.dumps(json.load(open('$O/bench.json'))['libgeeps_clock']))"; exit $rc
