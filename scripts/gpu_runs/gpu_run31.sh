#!/bin/bash
# Two HIP streams per channel (was five): libgeeps suite and end-to-end clocks
# at the default GPU_MAX_HW_QUEUES.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r31; mkdir -p $O/e2e
timeout -k 10 600 python -u -m pytest tests/test_libgeeps.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_libgeeps.log 2>&1; rc=$?
echo "libgeeps pytest rc=$rc"; tail -2 $O/pytest_libgeeps.log; [ $rc -eq 0 ] || exit $rc
run() { # name args...
  local name=$1; shift
  timeout -k 10 300 python scripts/run_clock_bench.py "$@" $O/e2e/$name.json > $O/e2e/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_clock_max": [0-9.]*' $O/e2e/$name.json 2>/dev/null)"; return $rc
}
run s2_t1Mx1024_1w_s0 1 8388608 10 2 0 ipc &&
run s2_t1Mx1024_2w_s0_ipc 2 8388608 10 2 0 ipc &&
run s2_alexnet_8w_s1_ipc 8 476292 20 3 1 ipc &&
run s2_alexnet_8w_s0_ipc 8 476292 20 3 0 ipc &&
run s2_t1Mx1024_8w_s0_ipc 8 8388608 6 2 0 ipc &&
run s2_alexnet_8w_s0_tcp 8 476292 10 2 0 tcp
