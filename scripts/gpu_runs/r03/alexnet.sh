#!/bin/bash
# Round 3: AlexNet-sized table, 8 worker processes on this GPU (configs[4]'s
# shape), standalone (no other GPU process), direct oplog on and off.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03alex}; mkdir -p $O
timeout -k 10 200 python scripts/run_clock_bench.py 8 476292 20 3 1 ipc $O/alexnet_8w_s1.json > /dev/null 2>> $O/err.txt || exit 1
GEEPS_DIRECT_OPLOG=0 timeout -k 10 200 python scripts/run_clock_bench.py 8 476292 20 3 1 ipc $O/alexnet_8w_s1_copy.json > /dev/null 2>> $O/err.txt || exit 1
timeout -k 10 200 python scripts/run_clock_bench.py 8 476292 20 3 0 ipc $O/alexnet_8w_s0.json > /dev/null 2>> $O/err.txt || exit 1
for f in $O/alexnet_*.json; do echo "$(basename $f) $(cat $f)"; done
