#!/bin/bash
# Phase-separated bucket sum in the product: parity, bench x3, per-allocation spread.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r40; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "bucket_sum or full_size or golden" > $O/pytest_sum.log 2>&1; rc=$?
echo "parity rc=$rc $(tail -1 $O/pytest_sum.log)"; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest_sum.log | head; exit $rc; }
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-inclusive --no-rowops > $O/bench_$i.json 2> $O/bench_$i.err; rc=$?
  echo "bench $i rc=$rc $(grep -o '"frac": [0-9.]*' $O/bench_$i.json | head -1) $(grep -o '"avg_kernel_ms": [0-9.]*' $O/bench_$i.json | head -1)"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 240 ./build/tune/alloc_tune 5 > $O/alloc.txt 2> $O/alloc.err; rc=$?
echo "alloc rc=$rc"; grep " sum" $O/alloc.txt; exit $rc
