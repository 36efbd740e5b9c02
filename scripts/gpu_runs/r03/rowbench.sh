#!/bin/bash
# Round 3: scan timings (probe 2) and the bench's row-op legs only.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03rowb}; mkdir -p $O
timeout -k 10 300 ./build/probe/r3_row_tune2 5 > $O/r3_row_tune2.txt 2> $O/r3_row_tune2.err; rc=$?
echo "probe rc=$rc"; head -14 $O/r3_row_tune2.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-inclusive --no-config2 --no-e2e --no-per-rank --no-pmc --no-separate-alloc > $O/bench_rowops.json 2> $O/bench_rowops.err; rc=$?
echo "bench rc=$rc"; exit $rc
