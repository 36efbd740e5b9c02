#!/bin/bash
# libgeeps after the tablet-server thread selects the process's device.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r28
timeout -k 10 600 python -u -m pytest tests/test_libgeeps.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r28/pytest_libgeeps.log 2>&1; rc=$?
echo "rc=$rc"; tail -3 gpurun_out/r28/pytest_libgeeps.log; exit $rc
