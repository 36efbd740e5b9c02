#!/bin/bash
# r05 dev16: where the 2-process libgeeps clock (1M x 1024 table as 8M
# RowData rows, configs[1]'s shape) spends its time: libgeeps timers, plus a
# kernel trace of the same run.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r05dev16}; mkdir -p $O
timeout -k 10 200 python -c "
import json, sys
sys.path.insert(0, 'scripts')
import run_clock_bench as m
r = m.run(2, 8388608, 10, 5, 0, 'ipc', timeout=120)
print(json.dumps({'ms_per_clock': r['ms_per_clock'], 'read_ok': r['read_ok'],
                  'client': [s['client'] for s in r['stats']], 'servers': [s['servers'] for s in r['stats']]}))
" > $O/p2_stats.json 2> $O/p2_stats.err; rc=$?
echo "rc=$rc $(head -c 200 $O/p2_stats.json)"; exit $rc
