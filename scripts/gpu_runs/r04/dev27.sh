#!/bin/bash
# Round 4: where the AlexNet-table clock's time goes with 8 processes on one
# GPU (slack 1): per-process client / server timers from the clock bench.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04dev27}; mkdir -p $O
timeout -k 10 200 python -c "
import json, sys
sys.path.insert(0, 'scripts')
import run_clock_bench as m
r = m.run(8, 476292, 20, 5, 1, 'ipc', timeout=150)
print(json.dumps({k: v for k, v in r.items() if k != 'probe'}))
" > $O/alex8.json 2> $O/alex8.err; rc=$?
echo "rc=$rc"; exit $rc
