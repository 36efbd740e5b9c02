#!/bin/bash
# Jittered (desynchronized) multi-process libgeeps tests.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r35; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_libgeeps.py -m gpu -x -v --timeout 300 --timeout-method thread -k jitter > $O/pytest_jitter.log 2>&1; rc=$?
echo "rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_jitter.log | tail -12; exit $rc
