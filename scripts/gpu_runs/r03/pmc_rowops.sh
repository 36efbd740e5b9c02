#!/bin/bash
# Round 3: PMC FETCH_SIZE / WRITE_SIZE passes (one counter per run) of the
# planned client row-op legs with the round-3 kernels, each leg alone in its run.
cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r03p; mkdir -p $O
B=$GRAFT_REPO_ROOT/bench.py
BASE="--no-cpu-baseline --no-host-inclusive --no-hbm-probe --no-config2 --no-e2e --no-per-rank --no-pmc --no-separate-alloc"
run() {  # name, bench args...
  local name=$1; shift
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_${name}_$c -o run -- python3 $B "$@" > $O/pmc_${name}_$c.log 2>&1; rc=$?
    echo "$name $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
}
for kind in random identity; do
  for leg in scatter_add_planned scatter_init_planned gather_planned; do
    run ${leg}_$kind $BASE --steps 1 --warmup 0 --rowops-only $leg --rowops-index $kind
  done
done
