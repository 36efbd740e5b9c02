#!/bin/bash
# End-to-end clocks with the phase-separated server sum.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r43; mkdir -p $O
run() { # name args...
  local name=$1; shift
  timeout -k 10 300 python scripts/run_clock_bench.py "$@" $O/$name.json > $O/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_clock_max": [0-9.]*' $O/$name.json 2>/dev/null)"; return $rc
}
true &&
true &&
run ph_t1Mx1024_8w_s0_ipc 8 8388608 6 2 0 ipc &&
run ph_alexnet_8w_s0_ipc 8 476292 20 3 0 ipc &&
run ph_alexnet_8w_s1_ipc 8 476292 20 3 1 ipc
