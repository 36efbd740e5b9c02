#!/bin/bash
# Round 2: per-rank work of the N = 1 / 2 / 4 / 8 bench, emulated on one GPU
# (bench.py --rows R/N: one rank's 8-bucket shard sum), current kernels.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r02m; mkdir -p $O
ARGS="--no-cpu-baseline --no-host-inclusive --no-rowops --no-e2e --no-config2 --no-hbm-probe --steps 20 --warmup 3"
for rep in 1 2; do
  for n in 1 2 4 8; do
    timeout -k 10 120 python bench.py $ARGS --rows $((1048576 / n)) > $O/emul_n${n}_r$rep.json 2> $O/emul_n${n}_r$rep.err; rc=$?
    echo "n=$n rep=$rep rc=$rc $(python3 -c "import json;d=json.load(open('$O/emul_n${n}_r$rep.json'));r=d['roofline'];print(d['ms_per_step'], r['frac'], r['launches_per_step'], r['other_launches_per_step'])")"; [ $rc -eq 0 ] || exit $rc
  done
done
