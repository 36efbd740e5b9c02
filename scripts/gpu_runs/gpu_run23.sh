#!/bin/bash
# Re-entry check of the rebuilt tree: full GPU suite, smoke, default bench line,
# and the rocprofv3 kernel-trace summary of the same bench command.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r23
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r23/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r23/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r23/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/r23/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/r23/bench.json 2> gpurun_out/r23/bench.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/r23/bench.json; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r23/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" > "$GRAFT_REPO_ROOT/gpurun_out/r23/prof_bench.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/r23/prof_bench.err"; rc=$?
echo "rocprof rc=$rc"; exit $rc
