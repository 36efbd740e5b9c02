#!/bin/bash
# Sweep kernel adopted: PMC FETCH/WRITE per launch at the 1/2/4/8-GPU shard sizes, rocprof kernel stats of the default bench, default bench, smoke.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r88; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1; rc=$?
echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err; rc=$?
echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
ARGS="--no-cpu-baseline --no-host-inclusive --no-rowops --no-hbm-probe --steps 2 --warmup 1"
for rows in 1048576 524288 262144 131072; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_${c}_$rows -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS --rows $rows > $O/pmc_${c}_$rows.log 2>&1; rc=$?
    echo "rows=$rows $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
