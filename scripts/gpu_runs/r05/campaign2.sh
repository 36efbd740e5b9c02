#!/bin/bash
# Round 5, after the shared host oplogs, the 16-MiB pieces and the host worker
# pool changed libgeeps' host side: the randomized libgeeps configurations
# (host tiers in 30 %, IPC faults in 20 % of them), 200 seeds.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r05campaign2}; mkdir -p $O
export PYTHONUNBUFFERED=1
GEEPS_STRESS_CASES=200 timeout -k 10 900 python -u -m pytest tests/test_libgeeps.py -m gpu -v -s -k "randomized" --timeout 250 --timeout-method thread > $O/pytest_stress.log 2>&1; rc=$?
echo "stress rc=$rc $(tail -n 1 $O/pytest_stress.log)"; grep -E "FAILED" $O/pytest_stress.log | head -20; exit $rc
