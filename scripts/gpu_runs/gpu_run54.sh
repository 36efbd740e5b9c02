#!/bin/bash
# Balanced form as its own instantiation (fixed forms compile-time again): suite, probe, e2e, bench.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r54; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "gpu suite rc=$rc $(tail -n 1 $O/pytest_gpu.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 ./build/tune/balance_tune 9 > $O/balance.txt 2> $O/balance.err; rc=$?
echo "balance rc=$rc"; [ $rc -eq 0 ] || exit $rc
run() { # name args...
  local name=$1; shift
  timeout -k 10 300 python scripts/run_clock_bench.py "$@" $O/$name.json > $O/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_clock_max": [0-9.]*' $O/$name.json 2>/dev/null)"; return $rc
}
run alexnet_8w_s0_ipc 8 476292 20 3 0 ipc &&
run alexnet_8w_s1_ipc 8 476292 20 3 1 ipc &&
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err; rc=$?
echo "bench rc=$rc $(grep -o '"frac": [0-9.]*' $O/bench_default.json | head -1) $(grep -o '"avg_kernel_ms": [0-9.]*' $O/bench_default.json | head -1)"; exit $rc
