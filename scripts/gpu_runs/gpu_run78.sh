#!/bin/bash
# Wave-map gather for every row size up to 128 floats: GPU suite, short-row probe, bench.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r78; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "gpu suite rc=$rc $(tail -n 1 $O/pytest_gpu.log)"; [ $rc -eq 0 ] || exit $rc
ROWMAP_SHORT=1 timeout -k 10 300 ./build/tune/rowmap_tune 7 > $O/short.txt 2> $O/short.err; rc=$?
echo "short rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err; rc=$?
echo "bench rc=$rc $(grep -o '"frac": [0-9.]*' $O/bench_default.json | tr '\n' ' ')"; exit $rc
