#!/bin/bash
# Round 3: random-row ceiling probe (probe 4) and the bench's row-op legs
# (with the repaired read-rate probe).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03rand}; mkdir -p $O
timeout -k 10 300 ./build/probe/r3_rand_tune 5 > $O/r3_rand_tune.txt 2> $O/r3_rand_tune.err; rc=$?
echo "probe rc=$rc"; cat $O/r3_rand_tune.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-inclusive --no-config2 --no-e2e --no-per-rank --no-pmc --no-separate-alloc > $O/bench_rowops.json 2> $O/bench_rowops.err; rc=$?
echo "bench rc=$rc"; exit $rc
