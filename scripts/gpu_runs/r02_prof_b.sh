#!/bin/bash
# Round 2: PMC FETCH_SIZE / WRITE_SIZE passes (one counter per run) for the
# 8-way sum, the 2-client sum (configs[1]) and every client row-op leg, each
# leg alone in its run so the kernel filter sees only that leg's dispatches.
cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r02p; mkdir -p $O
B=$GRAFT_REPO_ROOT/bench.py
BASE="--no-cpu-baseline --no-host-inclusive --no-hbm-probe --no-config2"
run() {  # name, bench args...
  local name=$1; shift
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_${name}_$c -o run -- python3 $B "$@" > $O/pmc_${name}_$c.log 2>&1; rc=$?
    echo "$name $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
}
run sum8 $BASE --no-rowops --steps 2 --warmup 1
run sum2 $BASE --no-rowops --steps 2 --warmup 1 --clients 2
for kind in random identity; do
  for leg in scatter_add scatter_add_planned scatter_init scatter_init_planned gather; do
    run ${leg}_$kind $BASE --steps 1 --warmup 0 --rowops-only $leg --rowops-index $kind
  done
done
