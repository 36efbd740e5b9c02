#!/bin/bash
# Kernel + memory-copy trace of the 2-worker 1M x 1024 end-to-end clock run.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/e2e
CLOCK_BENCH_PROF=$GRAFT_REPO_ROOT/gpurun_out/e2eprof timeout -k 10 400 python scripts/run_clock_bench.py 2 8388608 6 2 0 ipc gpurun_out/e2e/prof_2w.json > gpurun_out/e2e/prof_2w.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/e2e/prof_2w.log; exit $rc
