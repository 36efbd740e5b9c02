#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 30 --no-cpu-baseline --no-host-inclusive --no-rowops > gpurun_out/bench6_$i.json 2> gpurun_out/bench6_$i.err; rc=$?
  echo "bench $i rc=$rc $(grep -o '"avg_kernel_ms": [0-9.]*' gpurun_out/bench6_$i.json)"; [ $rc -eq 0 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof6" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 30 --no-cpu-baseline --no-host-inclusive --no-rowops > "$GRAFT_REPO_ROOT/gpurun_out/prof6.log" 2>&1; rc=$?
echo "rocprof rc=$rc $(grep -o '"avg_kernel_ms": [0-9.]*' $GRAFT_REPO_ROOT/gpurun_out/prof6.log)"
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --steps 30 --no-cpu-baseline --no-host-inclusive --no-rowops > gpurun_out/bench6_4.json 2> gpurun_out/bench6_4.err; rc=$?
echo "bench 4 rc=$rc $(grep -o '"avg_kernel_ms": [0-9.]*' gpurun_out/bench6_4.json)"
exit $rc
