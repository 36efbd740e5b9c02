#!/bin/bash
# Wave-map gather (LPR 32): GPU suite, probe, 1-worker e2e clock, default bench.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r76; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "gpu suite rc=$rc $(tail -n 1 $O/pytest_gpu.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 ./build/tune/rownt_tune 7 > $O/rownt.txt 2> $O/rownt.err; rc=$?
echo "rownt rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/run_clock_bench.py 1 8388608 10 2 0 ipc $O/t1Mx1024_1w_s0.json > $O/t1w.log 2>&1; rc=$?
echo "e2e 1w rc=$rc $(grep -o '"ms_per_clock_max": [0-9.]*' $O/t1Mx1024_1w_s0.json)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err; rc=$?
echo "bench rc=$rc $(grep -o '"frac": [0-9.]*' $O/bench_default.json | tr '\n' ' ')"; exit $rc
