#!/bin/bash
# Round 3: configs[4] (AlexNet blobs, 8 workers x 8 shards, slack 1) with and
# without direct reads.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03alexdread}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_libgeeps.py -m gpu -v -k "config5" --timeout 300 --timeout-method thread > $O/pytest_alex.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $O/pytest_alex.log)"; grep -E "FAILED|PASSED" $O/pytest_alex.log | head; exit $rc
