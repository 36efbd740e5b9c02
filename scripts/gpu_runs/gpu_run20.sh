#!/bin/bash
# libgeeps tests after the IPC key-part change, a traced 2-worker run, then e2e clock rates.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/e2e
timeout -k 10 600 python -m pytest tests/test_libgeeps.py -m gpu -q > gpurun_out/pytest20.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest20.log; [ $rc -eq 0 ] || exit $rc
CLOCK_BENCH_PROF=$GRAFT_REPO_ROOT/gpurun_out/e2eprof2 timeout -k 10 400 python scripts/run_clock_bench.py 2 8388608 6 2 0 ipc gpurun_out/e2e/prof2_2w.json > gpurun_out/e2e/prof2_2w.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -2 gpurun_out/e2e/prof2_2w.log; [ $rc -eq 0 ] || exit $rc
run() { # name args...
  local name=$1; shift
  timeout -k 10 400 python scripts/run_clock_bench.py "$@" gpurun_out/e2e/$name.json > gpurun_out/e2e/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/e2e/$name.log; return $rc
}
run r2_alexnet_8w_s1_ipc 8 476292 20 3 1 ipc &&
run r2_alexnet_8w_s0_ipc 8 476292 20 3 0 ipc &&
run r2_t1Mx1024_2w_s0_ipc 2 8388608 10 2 0 ipc &&
run r2_t1Mx1024_1w_s0 1 8388608 10 2 0 ipc
