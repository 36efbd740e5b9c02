#!/bin/bash
# Kernel + copy trace of the 1-process 4-GiB end-to-end clock (where the non-kernel time goes).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r62; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
CLOCK_BENCH_PROF=$O/prof timeout -k 10 300 python $GRAFT_REPO_ROOT/scripts/run_clock_bench.py 1 8388608 10 2 0 ipc $O/t1w.json > $O/t1w.log 2>&1; rc=$?
echo "e2e rc=$rc $(grep -o '"ms_per_clock_max": [0-9.]*' $O/t1w.json)"; exit $rc
