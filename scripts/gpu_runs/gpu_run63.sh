#!/bin/bash
# libgeeps multi-process tests against the host-UBSan build (scripts/build_ubsan.sh).
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r63; mkdir -p $O
GEEPS_SUM_APP=$GRAFT_REPO_ROOT/build/ubsan/geeps_sum_app timeout -k 10 900 python -u -m pytest tests/test_libgeeps.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_ubsan.log 2>&1; rc=$?
echo "ubsan libgeeps rc=$rc $(tail -n 1 $O/pytest_ubsan.log)"; grep -i "runtime error" -m 5 $O/pytest_ubsan.log; exit $rc
