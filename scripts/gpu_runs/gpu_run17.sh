#!/bin/bash
# GPU suite after the SHUTDOWN/ACK race fix, then the default bench line.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest17.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest17.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench17.json 2> gpurun_out/bench17.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench17.json; exit $rc
