#!/bin/bash
# Per-rank apply time of the N-GPU runs emulated on one GPU: the shard of R/N rows with 8 buckets.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r61; mkdir -p $O
ARGS="--no-cpu-baseline --no-host-inclusive --no-rowops --no-hbm-probe"
for rows in 1048576 524288 262144 131072; do
  timeout -k 10 300 python bench.py $ARGS --rows $rows --steps 40 > $O/bench_rows$rows.json 2> $O/bench_rows$rows.err; rc=$?
  echo "rows=$rows rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $O/bench_rows$rows.json) $(grep -o '"frac": [0-9.]*' $O/bench_rows$rows.json) $(grep -o '"launches_per_step": [0-9]*' $O/bench_rows$rows.json)"
  [ $rc -eq 0 ] || exit $rc
done
