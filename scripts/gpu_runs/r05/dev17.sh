#!/bin/bash
# r05 dev17: the host tier in plain (unpinned) host memory, as the
# reference keeps it (pinned_cpu_memory = 0), with the other host-tier tests.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r05dev17}; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_libgeeps.py -m gpu -v -k "host_tier" --timeout 150 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $O/pytest.log)"; grep FAILED $O/pytest.log | head; exit $rc
