#!/bin/bash
# Round 4: where the read-my-writes clock's time goes (2 processes, the
# 1M x 1024 table), kernel + copy trace per process.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04dev18}; mkdir -p $O
export TMPDIR=/tmp
CLOCK_BENCH_RMW=1 CLOCK_BENCH_PROF=$O/prof timeout -k 10 300 python scripts/run_clock_bench.py 2 8388608 5 2 0 ipc > $O/rmw_prof.json 2> $O/rmw_prof.err; rc=$?
echo "rmw prof rc=$rc"; cat $O/rmw_prof.json; exit $rc
