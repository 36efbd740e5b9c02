#!/bin/bash
# Phased sum at 160 KiB of LDS per block, 1 block/CU, 2 chunks/launch:
# full GPU suite, default bench, rocprof summary, FETCH/WRITE passes, K / block-size probe.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r45; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "gpu suite rc=$rc $(tail -n 1 $O/pytest_gpu.log)"; [ $rc -eq 0 ] || exit $rc
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
timeout -k 10 300 ./build/tune/phase_tune 5 4 > $O/phase.txt 2> $O/phase.err; rc=$?
echo "phase rc=$rc"; exit $rc
