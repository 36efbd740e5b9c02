#!/bin/bash
# End-to-end clocks with GPU_MAX_HW_QUEUES=2 per process, so that P processes on
# the box's ONE GPU do not oversubscribe its hardware queues (one process per
# GPU on an 8-GPU node never does).
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r32; mkdir -p $O
export GPU_MAX_HW_QUEUES=2
run() { # name args...
  local name=$1; shift
  timeout -k 10 300 python scripts/run_clock_bench.py "$@" $O/$name.json > $O/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_clock_max": [0-9.]*' $O/$name.json 2>/dev/null)"; return $rc
}
run hq2_t1Mx1024_1w_s0 1 8388608 10 2 0 ipc &&
run hq2_t1Mx1024_2w_s0_ipc 2 8388608 10 2 0 ipc &&
run hq2_t1Mx1024_8w_s0_ipc 8 8388608 6 2 0 ipc &&
run hq2_alexnet_8w_s0_ipc 8 476292 20 3 0 ipc &&
run hq2_alexnet_8w_s1_ipc 8 476292 20 3 1 ipc &&
run hq2_alexnet_8w_s0_tcp 8 476292 10 2 0 tcp &&
run hq2_t128M_2w_s0_tcp 2 262144 10 2 0 tcp
