#!/bin/bash
# Round 2: bench with the per-rank emulation leg (side legs off).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r02pr; mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-inclusive --no-rowops --no-e2e > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['ms_per_step'], json.dumps(d.get('per_rank_emulation')))"; [ $rc -eq 0 ] || { tail -20 $O/bench.err; exit $rc; }
