#!/bin/bash
# First GPU pass: smoke -> bench -> gpu tests -> rocprof kernel trace.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
stop() { echo "STOP rc=$1 at $2"; exit "$1"; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; [ $rc -eq 0 ] || stop $rc smoke
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/bench1.json 2> gpurun_out/bench1.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench1.json; [ $rc -eq 0 ] || stop $rc bench
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then stop $rc pytest; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof1" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-host-inclusive > "$GRAFT_REPO_ROOT/gpurun_out/prof1.log" 2>&1; rc=$?
echo "rocprof rc=$rc"
exit 0
