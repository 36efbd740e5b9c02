#!/bin/bash
# r05 dev18: kernel trace of the 2-process libgeeps clock on the 4-GiB table
# (how much of each clock the GPU is busy), rocprofv3 over the driver script
# and its two app processes.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r05dev18}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -c "
import json, sys
sys.path.insert(0, '$GRAFT_REPO_ROOT/scripts')
import run_clock_bench as m
r = m.run(2, 8388608, 10, 5, 0, 'ipc', timeout=200)
print(json.dumps({'ms_per_clock': r['ms_per_clock'], 'read_ok': r['read_ok']}))
" > $O/p2_trace.json 2> $O/p2_trace.err; rc=$?
echo "rc=$rc $(cat $O/p2_trace.json | head -c 300)"; ls -R $O/prof | head -20; exit $rc
