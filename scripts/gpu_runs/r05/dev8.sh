#!/bin/bash
# r05 dev8: where the host tier's clock goes (libgeeps timers), AlexNet-sized
# table, half of its rows in the host tier, 2 processes.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r05dev8}; mkdir -p $O
timeout -k 10 200 python -c "
import json, sys
sys.path.insert(0, 'scripts')
import run_clock_bench as m
r = m.run(2, 476292, 10, 5, 0, 'ipc', timeout=120, extra_env={'CLOCK_BENCH_HOST_TIER_FRAC': '0.5'})
print(json.dumps({'ms_per_clock': r['ms_per_clock'], 'read_ok': r['read_ok'],
                  'client': [s['client'] for s in r['stats']], 'servers': [s['servers'] for s in r['stats']]}))
" > $O/host_tier_stats.json 2> $O/host_tier_stats.err; rc=$?
echo "rc=$rc"; cat $O/host_tier_stats.json; exit $rc
