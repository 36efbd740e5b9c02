#!/bin/bash
# Round 2: PMC of the planned identity row-op legs (their dense runs through
# the sweep kernels, whose names now carry the tile width).
cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r02pp; mkdir -p $O
B=$GRAFT_REPO_ROOT/bench.py
BASE="--no-cpu-baseline --no-host-inclusive --no-hbm-probe --no-config2 --no-e2e --no-per-rank --steps 1 --warmup 0"
run() {  # name, bench args...
  local name=$1; shift
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_${name}_$c -o run -- python3 $B "$@" > $O/pmc_${name}_$c.log 2>&1; rc=$?
    echo "$name $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
}
for leg in scatter_add_planned scatter_init_planned gather_planned; do
  run ${leg}_identity $BASE --rowops-only $leg --rowops-index identity
done
