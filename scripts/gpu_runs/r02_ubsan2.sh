#!/bin/bash
# Round 2: host UBSan pass of libgeeps after the gather plans (every
# multi-process libgeeps case), then smoke.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r02u; mkdir -p $O
GEEPS_SUM_APP=build/ubsan/geeps_sum_app timeout -k 10 900 python -u -m pytest tests/test_libgeeps.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_ubsan.log 2>&1; rc=$?
echo "ubsan pytest rc=$rc $(tail -n 1 $O/pytest_ubsan.log)"; [ $rc -eq 0 ] || { grep -E "runtime error|FAIL" $O/pytest_ubsan.log | head; exit $rc; }
grep -c "runtime error" $O/pytest_ubsan.log || true
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; rc=$?
echo "smoke rc=$rc $(tail -n 1 $O/smoke.txt)"; exit $rc
