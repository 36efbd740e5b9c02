#!/bin/bash
# Round 4: randomized libgeeps configurations (processes, slack, channels,
# tables, read-my-writes, local access, transport, layers, shuffles, jitter,
# direct oplog, staging switches), every Read checked by the app.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04stress}; mkdir -p $O
GEEPS_STRESS_CASES=${2:-60} timeout -k 10 1000 python -u -m pytest tests/test_libgeeps.py -m gpu -v -s -k "randomized" --timeout 250 --timeout-method thread > $O/pytest_stress.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $O/pytest_stress.log)"; grep -E "FAILED" $O/pytest_stress.log | head -20; exit $rc
