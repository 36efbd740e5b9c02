#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2 3; do
  for L in arena separate; do
    timeout -k 10 200 python bench.py --steps 20 --layout $L --no-cpu-baseline --no-host-inclusive --no-rowops > gpurun_out/ab_${L}_$i.json 2> gpurun_out/ab_${L}_$i.err; rc=$?
    echo "$L $i rc=$rc $(grep -o '"avg_kernel_ms": [0-9.]*' gpurun_out/ab_${L}_$i.json) $(grep -o '"frac": [0-9.]*' gpurun_out/ab_${L}_$i.json | head -1)"
    [ $rc -eq 0 ] || exit $rc
  done
done
