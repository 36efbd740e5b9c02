#!/bin/bash
# AlexNet-table 8-process clock: does hardware-queue oversubscription (8 processes
# x GPU_MAX_HW_QUEUES queues on one GPU) set the per-clock time?
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r30; mkdir -p $O
run() { # name args...
  local name=$1; shift
  timeout -k 10 300 python scripts/run_clock_bench.py "$@" $O/$name.json > $O/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_clock_max": [0-9.]*' $O/$name.json 2>/dev/null)"; return $rc
}
run q4_alex_s0 8 476292 20 3 0 ipc &&
GPU_MAX_HW_QUEUES=2 run q2_alex_s0 8 476292 20 3 0 ipc &&
GPU_MAX_HW_QUEUES=1 run q1_alex_s0 8 476292 20 3 0 ipc &&
run q4_alex_2w_s0 2 476292 20 3 0 ipc &&
run q4_alex_4w_s0 4 476292 20 3 0 ipc
