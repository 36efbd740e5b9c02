#!/bin/bash
# r05: libgeeps under UBSan (host code only; scripts/build_ubsan.sh): the tests
# of this round's host code (IPC recovery, host tier, swap), plus 40
# randomized configurations.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r05ubsan}; mkdir -p $O
export PYTHONUNBUFFERED=1
GEEPS_SUM_APP=$GRAFT_REPO_ROOT/build/ubsan/geeps_sum_app GEEPS_STRESS_CASES=40 timeout -k 10 600 python -u -m pytest tests/test_libgeeps.py -m gpu -v -k "host_tier or ipc_failure or randomized or peer_refresh or read_my_writes or tcp" --timeout 175 --timeout-method thread > $O/pytest_ubsan.log 2>&1; rc=$?
echo "ubsan rc=$rc $(tail -n 1 $O/pytest_ubsan.log)"; grep -E "FAILED|runtime error" $O/pytest_ubsan.log | head; exit $rc
