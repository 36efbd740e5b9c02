#!/bin/bash
# Round 4: socket pushes and replies sent in pieces as their D2H lands: the
# libgeeps tests (TCP cases, randomized mixes), then the loopback-TCP clock.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04dev21}; mkdir -p $O
GEEPS_STRESS_CASES=60 timeout -k 10 600 python -u -m pytest tests/test_libgeeps.py -m gpu -v --timeout 175 --timeout-method thread > $O/pytest_libgeeps.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $O/pytest_libgeeps.log)"; grep -E "FAILED" $O/pytest_libgeeps.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/run_clock_bench.py 2 476292 10 2 0 tcp > $O/tcp.json 2> $O/tcp.err; rc=$?
echo "tcp rc=$rc"; cat $O/tcp.json; exit $rc
