#!/bin/bash
# Phased sum with non-temporal master accesses and 2 chunks/launch at 8 buckets:
# parity, default bench, headline rocprof summary, FETCH/WRITE passes, alloc spread.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r44; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_parity.log 2>&1; rc=$?
echo "parity rc=$rc $(tail -1 $O/pytest_parity.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err; rc=$?
echo "bench rc=$rc $(grep -o '"frac": [0-9.]*' $O/bench_default.json | head -1) $(grep -o '"avg_kernel_ms": [0-9.]*' $O/bench_default.json | head -1)"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu-baseline --no-host-inclusive --no-rowops --no-hbm-probe"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $O/prof_bench.json 2> $O/prof_bench.err; rc=$?
echo "rocprof rc=$rc $(grep -o '"avg_launch_ms": [0-9.]*' $O/prof_bench.json)"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS --steps 2 --warmup 1 > $O/pmc_fetch.log 2>&1; rc=$?
echo "pmc fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS --steps 2 --warmup 1 > $O/pmc_write.log 2>&1; rc=$?
echo "pmc write rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $GRAFT_REPO_ROOT
timeout -k 10 240 ./build/tune/alloc_tune 5 > $O/alloc.txt 2> $O/alloc.err; rc=$?
echo "alloc rc=$rc"; grep " sum" $O/alloc.txt; exit $rc
