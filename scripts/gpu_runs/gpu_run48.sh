#!/bin/bash
# End-to-end clocks and the 2-client config line with the 160-KiB phased server sum.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r48; mkdir -p $O
run() { # name args...
  local name=$1; shift
  timeout -k 10 300 python scripts/run_clock_bench.py "$@" $O/$name.json > $O/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_clock_max": [0-9.]*' $O/$name.json 2>/dev/null)"; return $rc
}
run t1Mx1024_1w_s0 1 8388608 10 2 0 ipc &&
run t1Mx1024_2w_s0_ipc 2 8388608 10 2 0 ipc &&
run t1Mx1024_8w_s0_ipc 8 8388608 6 2 0 ipc &&
run alexnet_8w_s0_ipc 8 476292 20 3 0 ipc &&
run alexnet_8w_s1_ipc 8 476292 20 3 1 ipc &&
timeout -k 10 300 python bench.py --clients 2 --no-host-inclusive --no-rowops > $O/bench_2clients.json 2> $O/bench_2clients.err; rc=$?
echo "bench 2 clients rc=$rc $(grep -o '"frac": [0-9.]*' $O/bench_2clients.json | head -1) $(grep -o '"avg_kernel_ms": [0-9.]*' $O/bench_2clients.json | head -1)"; exit $rc
