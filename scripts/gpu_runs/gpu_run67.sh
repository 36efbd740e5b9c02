#!/bin/bash
# FETCH/WRITE per launch of the 2/4/8-GPU runs' shard sums, on one GPU (bench --rows R/N).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r67; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu-baseline --no-host-inclusive --no-rowops --no-hbm-probe --steps 2 --warmup 1"
for rows in 524288 262144 131072; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_${c}_$rows -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS --rows $rows > $O/pmc_${c}_$rows.log 2>&1; rc=$?
    echo "rows=$rows $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
