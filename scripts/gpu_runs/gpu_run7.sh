#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1000 python -m pytest tests/test_libgeeps.py -m gpu -q -x --durations=10 > gpurun_out/pytest_libgeeps7.log 2>&1; rc=$?
echo "libgeeps pytest rc=$rc"; tail -30 gpurun_out/pytest_libgeeps7.log
exit $rc
