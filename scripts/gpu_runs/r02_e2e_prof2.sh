#!/bin/bash
# Round 2: kernel trace of the 1-process libgeeps clock (4 GiB table) with the (bursts-of-2) current kernels, gather plans and
# current kernels.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r02t2; mkdir -p $O
export TMPDIR=/tmp
CLOCK_BENCH_PROF=$O/prof timeout -k 10 300 python scripts/run_clock_bench.py 1 8388608 10 2 0 ipc $O/t4g_1w_prof.json > $O/run.log 2>&1; rc=$?
echo "rc=$rc"; cat $O/t4g_1w_prof.json; exit $rc
