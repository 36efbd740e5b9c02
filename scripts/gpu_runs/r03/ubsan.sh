#!/bin/bash
# Round 3: the libgeeps GPU tests with the host-UBSan build of libgeeps and the
# sum app (scripts/build_ubsan.sh): ZMTP transport, direct oplog, staging.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03ubsan}; mkdir -p $O
GEEPS_SUM_APP=$GRAFT_REPO_ROOT/build/ubsan/geeps_sum_app timeout -k 10 700 python -u -m pytest tests/test_libgeeps.py -m gpu -v --timeout 175 --timeout-method thread > $O/pytest_ubsan.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $O/pytest_ubsan.log)"; grep -E "FAILED|runtime error" $O/pytest_ubsan.log | head -20; exit $rc
