#!/bin/bash
# Round 3: the cached-plan compare fast path -- every GPU parity test (fuzzed
# unplanned calls widened to 200 cases), then the default bench.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03cmp}; mkdir -p $O
GEEPS_FUZZ_CASES=200 timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 175 --timeout-method thread > $O/pytest_parity.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $O/pytest_parity.log)"; grep -E "FAILED" $O/pytest_parity.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > $O/bench_default.json 2> $O/bench_default.err; rc=$?
echo "bench rc=$rc"; exit $rc
