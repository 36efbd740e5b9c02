#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 ./scripts/tune/bucket_tune $((1<<20)) 1024 8 7 > gpurun_out/tune8.txt 2> gpurun_out/tune8.err; rc=$?
echo "tune rc=$rc"; cat gpurun_out/tune8.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke16.log 2>&1; rc=$?
echo "smoke rc=$rc"; cat gpurun_out/smoke16.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest16.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest16.log; exit $rc
