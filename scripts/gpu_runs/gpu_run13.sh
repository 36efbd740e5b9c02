#!/bin/bash
# Full default bench + its rocprof kernel-trace summary + PMC traffic passes.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench13.json 2> gpurun_out/bench13.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench13.json; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof13" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --no-host-inclusive > "$GRAFT_REPO_ROOT/gpurun_out/prof13.log" 2>&1; rc=$?
echo "rocprof rc=$rc $(grep -o '"avg_kernel_ms": [0-9.]*' $GRAFT_REPO_ROOT/gpurun_out/prof13.log | head -1)"; [ $rc -eq 0 ] || exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc13_$c" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-host-inclusive > "$GRAFT_REPO_ROOT/gpurun_out/pmc13_$c.log" 2>&1; rc=$?
  echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
