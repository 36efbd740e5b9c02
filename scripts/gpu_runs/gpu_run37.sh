#!/bin/bash
# Jittered libgeeps tests, three passes (host-side concurrency check), then the whole libgeeps suite.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r37; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 600 python -u -m pytest tests/test_libgeeps.py -m gpu -x -v --timeout 300 --timeout-method thread -k jitter > $O/pytest_jitter_$i.log 2>&1; rc=$?
  echo "pass $i rc=$rc $(tail -1 $O/pytest_jitter_$i.log)"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 900 python -u -m pytest tests/test_libgeeps.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_libgeeps.log 2>&1; rc=$?
echo "suite rc=$rc $(tail -1 $O/pytest_libgeeps.log)"; exit $rc
