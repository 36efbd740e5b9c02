#!/bin/bash
# Round 3: probe 2 (scan v2, hipCUB sort, contiguous buffers), then the libgeeps
# GPU tests verbosely (a 2-process run hung in r03base).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r03libg; mkdir -p $O
timeout -k 10 300 ./build/probe/r3_row_tune2 7 > $O/r3_row_tune2.txt 2> $O/r3_row_tune2.err; rc=$?
echo "probe rc=$rc"; cat $O/r3_row_tune2.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests/test_libgeeps.py -m gpu -v --timeout 170 --timeout-method thread > $O/pytest_libgeeps.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" $O/pytest_libgeeps.log | tail -20; exit $rc
