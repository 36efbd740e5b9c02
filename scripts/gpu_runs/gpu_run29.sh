#!/bin/bash
# Zero-copy refresh (servers publish master versions, clients read them in place):
# out-of-place sum parity, libgeeps suite, end-to-end clock rates.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r29; mkdir -p $O/e2e
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "bucket_sum" > $O/pytest_sum.log 2>&1; rc=$?
echo "sum pytest rc=$rc"; tail -2 $O/pytest_sum.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_libgeeps.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_libgeeps.log 2>&1; rc=$?
echo "libgeeps pytest rc=$rc"; tail -4 $O/pytest_libgeeps.log; [ $rc -eq 0 ] || exit $rc
run() { # name args...
  local name=$1; shift
  timeout -k 10 300 python scripts/run_clock_bench.py "$@" $O/e2e/$name.json > $O/e2e/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc $(cut -c1-200 $O/e2e/$name.json 2>/dev/null)"; return $rc
}
run v_t1Mx1024_1w_s0 1 8388608 10 2 0 ipc &&
run v_t1Mx1024_2w_s0_ipc 2 8388608 10 2 0 ipc &&
run v_alexnet_8w_s1_ipc 8 476292 20 3 1 ipc &&
run v_alexnet_8w_s0_ipc 8 476292 20 3 0 ipc &&
run v_t1Mx1024_8w_s0_ipc 8 8388608 6 2 0 ipc
