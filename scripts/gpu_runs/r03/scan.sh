#!/bin/bash
# Round 3: the unplanned calls' overhead: probe 2 (scan / compare / D2H / sync in
# isolation) and a kernel trace of the bench's row-op legs.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r03scan; mkdir -p $O
timeout -k 10 300 ./build/probe/r3_row_tune2 7 > $O/r3_row_tune2b.txt 2> $O/r3_row_tune2b.err; rc=$?
echo "probe rc=$rc"; cat $O/r3_row_tune2b.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-inclusive --no-hbm-probe --no-config2 --no-e2e --no-per-rank --no-pmc --no-separate-alloc > $O/prof_bench.json 2> $O/prof_bench.err; rc=$?
echo "rocprof rc=$rc"; exit $rc
