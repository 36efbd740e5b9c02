#!/bin/bash
# Round 2: bench with the libgeeps leg only (1, 2 and 8 processes), other side legs off.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r02e4; mkdir -p $O
timeout -k 10 400 python bench.py --no-cpu-baseline --no-host-inclusive --no-rowops --steps 5 > $O/bench_e2e.json 2> $O/bench_e2e.err; rc=$?
echo "bench rc=$rc"; python3 -c "import json; d=json.load(open('$O/bench_e2e.json')); print(json.dumps(d.get('libgeeps_clock')))"; [ $rc -eq 0 ] || { tail -20 $O/bench_e2e.err; exit $rc; }
