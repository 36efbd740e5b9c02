#!/bin/bash
# nt loads of the op buffer in scatter-add / fused init: GPU suite, probe A/B, default bench (row-op leg).
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r58; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "gpu suite rc=$rc $(tail -n 1 $O/pytest_gpu.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 ./build/tune/rownt_tune 7 > $O/rownt.txt 2> $O/rownt.err; rc=$?
echo "rownt rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err; rc=$?
echo "bench rc=$rc $(grep -o '"frac": [0-9.]*' $O/bench_default.json | tr '\n' ' ')"; exit $rc
