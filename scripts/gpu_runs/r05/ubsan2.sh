#!/bin/bash
# r05: libgeeps under UBSan (host code only; scripts/build_ubsan.sh) at the
# final code: host tier (shared oplogs, pieces, fused init, runs), IPC
# recovery, rehearsal and 60 randomized configurations.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r05ubsan2}; mkdir -p $O
export PYTHONUNBUFFERED=1
GEEPS_SUM_APP=$GRAFT_REPO_ROOT/build/ubsan/geeps_sum_app GEEPS_STRESS_CASES=60 timeout -k 10 700 python -u -m pytest tests/test_libgeeps.py -m gpu -v -k "host_tier or ipc_failure or randomized or rehearsal" --timeout 175 --timeout-method thread > $O/pytest_ubsan.log 2>&1; rc=$?
echo "ubsan rc=$rc $(tail -n 1 $O/pytest_ubsan.log)"; grep -E "FAILED|runtime error" $O/pytest_ubsan.log | head; exit $rc
