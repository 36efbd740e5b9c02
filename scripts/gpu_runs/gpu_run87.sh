#!/bin/bash
# Sweep form at 6 register tiles, bursts of 4 (scheduling fixed): A/B against the tile-major plan and other shapes, GPU suite, default bench.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r87; mkdir -p $O
timeout -k 10 400 ./build/tune/bmaj_tune 7 3 > $O/sweep_ab2.txt 2> $O/ab.err; rc=$?
echo "ab rc=$rc"; cat $O/sweep_ab2.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "gpu suite rc=$rc $(tail -n 1 $O/pytest_gpu.log)"; [ $rc -eq 0 ] || { tail -30 $O/pytest_gpu.log; exit $rc; }
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err; rc=$?
echo "bench rc=$rc"; cat $O/bench_default.json | head -c 1500; exit $rc
