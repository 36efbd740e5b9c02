#!/bin/bash
# Round 2: bench with the libgeeps end-to-end clock leg (other side legs off),
# then PMC FETCH_SIZE / WRITE_SIZE passes of the N = 2 / 4 / 8 per-rank shard
# sums (one rank's work on one GPU: --rows R/N), refreshed on the sweep kernel.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r02e; mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-inclusive --no-rowops --steps 5 > $O/bench_e2e.json 2> $O/bench_e2e.err; rc=$?
echo "bench rc=$rc"; cat $O/bench_e2e.json | python3 -c "import json,sys; d=json.load(sys.stdin); print(json.dumps(d.get('libgeeps_clock')))"; [ $rc -eq 0 ] || { tail -20 $O/bench_e2e.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp
B=$GRAFT_REPO_ROOT/bench.py
BASE="--no-cpu-baseline --no-host-inclusive --no-hbm-probe --no-config2 --no-rowops --no-e2e --steps 2 --warmup 1"
for n in 2 4 8; do
  rows=$((1048576 / n))
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_g${n}_$c -o run -- python3 $B $BASE --rows $rows > $O/pmc_g${n}_$c.log 2>&1; rc=$?
    echo "g$n $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
