#!/bin/bash
# Segmented-cache kernels + in-place IPC refresh: parity, libgeeps, e2e clock rates.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/e2e
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -q -k "segmented or golden" > gpurun_out/pytest21a.log 2>&1; rc=$?
echo "seg pytest rc=$rc"; tail -3 gpurun_out/pytest21a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -m pytest tests/test_libgeeps.py -m gpu -q > gpurun_out/pytest21b.log 2>&1; rc=$?
echo "libgeeps pytest rc=$rc"; tail -3 gpurun_out/pytest21b.log; [ $rc -eq 0 ] || exit $rc
run() { # name args...
  local name=$1; shift
  timeout -k 10 400 python scripts/run_clock_bench.py "$@" gpurun_out/e2e/$name.json > gpurun_out/e2e/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/e2e/$name.log; return $rc
}
run r3_t1Mx1024_2w_s0_ipc 2 8388608 10 2 0 ipc &&
run r3_alexnet_8w_s1_ipc 8 476292 20 3 1 ipc &&
run r3_alexnet_8w_s0_ipc 8 476292 20 3 0 ipc &&
run r3_t1Mx1024_8w_s0_ipc 8 8388608 6 2 0 ipc
