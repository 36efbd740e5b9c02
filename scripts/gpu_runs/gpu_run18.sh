#!/bin/bash
# End-to-end libgeeps clock rates through the public API (scripts/run_clock_bench.py):
# configs[4] AlexNet-sized table (476,292 RowData rows) with 8 workers x 8 shards at
# staleness 1 over both transports, and the 1M x 1024 table (8,388,608 rows) with 2 workers.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/e2e
run() { # name args...
  local name=$1; shift
  timeout -k 10 400 python scripts/run_clock_bench.py "$@" gpurun_out/e2e/$name.json > gpurun_out/e2e/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; cat gpurun_out/e2e/$name.log | tail -3; return $rc
}
run alexnet_8w_s1_ipc 8 476292 20 3 1 ipc &&
run alexnet_8w_s1_tcp 8 476292 10 2 1 tcp &&
run alexnet_8w_s0_ipc 8 476292 20 3 0 ipc &&
run t1Mx1024_2w_s0_ipc 2 8388608 10 2 0 ipc &&
run t1Mx1024_8w_s0_ipc 8 8388608 6 2 0 ipc
