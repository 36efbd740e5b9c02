#!/bin/bash
# Round 3: direct read with one Read op per server shard -- the clock bench at
# 2 workers (4 GiB table) and the AlexNet-sized table at 8 workers, slack 1,
# with direct reads on and off.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03dread2}; mkdir -p $O
export CLOCK_BENCH_READ_PER_SHARD=1
for i in 1 2; do
  timeout -k 10 200 python scripts/run_clock_bench.py 2 8388608 10 2 0 ipc $O/clock_p2_shardreads_gather_$i.json > /dev/null 2>> $O/clock.err || exit 1
  GEEPS_DIRECT_READ=1 timeout -k 10 200 python scripts/run_clock_bench.py 2 8388608 10 2 0 ipc $O/clock_p2_shardreads_direct_$i.json > /dev/null 2>> $O/clock.err || exit 1
  timeout -k 10 200 python scripts/run_clock_bench.py 8 476292 10 2 1 ipc $O/clock_p8_alexnet_shardreads_gather_$i.json > /dev/null 2>> $O/clock.err || exit 1
  GEEPS_DIRECT_READ=1 timeout -k 10 200 python scripts/run_clock_bench.py 8 476292 10 2 1 ipc $O/clock_p8_alexnet_shardreads_direct_$i.json > /dev/null 2>> $O/clock.err || exit 1
done
for f in $O/clock_*.json; do echo "$(basename $f) $(python -c "import json,sys; d=json.load(open('$f')); print(d['ms_per_clock_max'], d['ms_per_clock'])")"; done
