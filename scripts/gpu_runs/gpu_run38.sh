#!/bin/bash
# Lazy param cache (not allocated when every refresh is read in place) + empty-setup tests.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r38; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_libgeeps.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_libgeeps.log 2>&1; rc=$?
echo "suite rc=$rc $(tail -1 $O/pytest_libgeeps.log)"; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_libgeeps.log | head -20; exit $rc; }
timeout -k 10 300 python scripts/run_clock_bench.py 1 8388608 10 2 0 ipc $O/lazy_1w.json > $O/lazy_1w.log 2>&1; rc=$?
echo "1w rc=$rc $(grep -o '"ms_per_clock_max": [0-9.]*' $O/lazy_1w.json)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/run_clock_bench.py 8 8388608 6 2 0 ipc $O/lazy_8w.json > $O/lazy_8w.log 2>&1; rc=$?
echo "8w rc=$rc $(grep -o '"ms_per_clock_max": [0-9.]*' $O/lazy_8w.json)"; exit $rc
