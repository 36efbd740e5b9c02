#!/bin/bash
# Round 2: end-to-end libgeeps clock (public API) after the row plans and the
# wave-map scatter forms: 1 / 2 / 8 processes on the 4-GiB table, 8 on the
# AlexNet table (BSP, staleness 1), and 2 processes with peer-bucket staging
# forced (the cross-GPU path's copy + local sum, on one GPU).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r02e; mkdir -p $O
run() { # name args...
  local name=$1; shift
  timeout -k 10 300 python scripts/run_clock_bench.py "$@" $O/$name.json > $O/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_clock_max": [0-9.]*' $O/$name.json 2>/dev/null)"; return $rc
}
run t4g_1w 1 8388608 10 2 0 ipc &&
run t4g_2w 2 8388608 8 2 0 ipc &&
run t4g_8w 8 8388608 6 2 0 ipc &&
run alexnet_8w_s0_ipc 8 476292 20 3 0 ipc &&
run alexnet_8w_s1_ipc 8 476292 20 3 1 ipc &&
GEEPS_STAGE_PEER_UPDATES=1 run t4g_2w_staged 2 8388608 8 2 0 ipc
