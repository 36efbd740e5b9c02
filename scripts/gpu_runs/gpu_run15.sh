#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_libgeeps.py -m gpu -q -x > gpurun_out/pytest15.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -25 gpurun_out/pytest15.log; exit $rc
