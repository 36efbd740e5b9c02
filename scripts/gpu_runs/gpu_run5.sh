#!/bin/bash
# Row-op sweep, then the bench with its rocprof kernel-trace summary and PMC traffic passes.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 ./scripts/tune/rowop_tune $((1<<23)) 5 > gpurun_out/rowtune1.txt 2> gpurun_out/rowtune1.err; rc=$?
echo "rowtune rc=$rc"; cat gpurun_out/rowtune1.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench5.json 2> gpurun_out/bench5.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench5.json; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof5" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --no-host-inclusive > "$GRAFT_REPO_ROOT/gpurun_out/prof5.log" 2>&1; rc=$?
echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc5_$c" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-host-inclusive > "$GRAFT_REPO_ROOT/gpurun_out/pmc5_$c.log" 2>&1; rc=$?
  echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
