#!/bin/bash
# Round 3: the row-op probe (scripts/tune/r3_row_tune.hip), GPU suite, default bench.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r03base; mkdir -p $O
timeout -k 10 300 ./build/probe/r3_row_tune 7 > $O/r3_row_tune.txt 2> $O/r3_row_tune.err; rc=$?
echo "probe rc=$rc"; cat $O/r3_row_tune.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $O/pytest_gpu.log)"; grep -E "FAILED|passed,|failed," $O/pytest_gpu.log | head -20
timeout -k 10 500 python bench.py > $O/bench_default.json 2> $O/bench_default.err; rc=$?
echo "bench rc=$rc"; exit $rc
