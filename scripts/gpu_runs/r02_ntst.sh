#!/bin/bash
# Round 2: non-temporal oplog stores for the op-order scatter-add (2 blocks per CU): GPU
# suite, smoke, default bench, rocprof stats, PMC of the unplanned scatter-add
# legs (random and identity index).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r02ntst; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $O/pytest_gpu.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1; rc=$?
echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > $O/bench_default.json 2> $O/bench_default.err; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/bench_default.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp
B=$GRAFT_REPO_ROOT/bench.py
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $B --no-cpu-baseline --no-host-inclusive --no-e2e > $O/prof_bench.json 2> $O/prof_bench.err; rc=$?
echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
BASE="--no-cpu-baseline --no-host-inclusive --no-hbm-probe --no-config2 --no-e2e --no-per-rank"
run() {  # name, bench args...
  local name=$1; shift
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_${name}_$c -o run -- python3 $B "$@" > $O/pmc_${name}_$c.log 2>&1; rc=$?
    echo "$name $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
}
for kind in random identity; do
  run scatter_add_$kind $BASE --steps 1 --warmup 0 --rowops-only scatter_add --rowops-index $kind
done
