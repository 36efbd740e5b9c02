#!/bin/bash
# Round 4: the zero-bucket copy through the sweep kernels and the fused
# read-my-writes refresh: their tests, then the rmw clock again.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04dev19}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_libgeeps.py -m gpu -v -k "bucket_sum_into or test_libgeeps" --timeout 175 --timeout-method thread > $O/pytest_rmw.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $O/pytest_rmw.log)"; grep -E "FAILED" $O/pytest_rmw.log | head; [ $rc -eq 0 ] || exit $rc
CLOCK_BENCH_RMW=1 timeout -k 10 200 python scripts/run_clock_bench.py 2 8388608 10 2 0 ipc > $O/rmw.json 2> $O/rmw.err; rc=$?
echo "rmw rc=$rc"; cat $O/rmw.json; exit $rc
