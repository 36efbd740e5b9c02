#!/bin/bash
# Round 6: the 300-seed randomized libgeeps campaign with every process's IPC
# audit log (GEEPS_IPC_LOG), then scripts/ipc_audit.py over them.  Run twice,
# once per build: "before" (a mis-mapping unmapped again, a replaced oplog
# buffer's mapping closed at once) and "after" (both kept mapped until
# Shutdown, so no address that held a mapping is reused by an export).
set -u
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r06/${1:-campaign}; mkdir -p $O
export PYTHONUNBUFFERED=1
GEEPS_STRESS_CASES=300 GEEPS_IPC_LOG=1 GEEPS_TEST_LOG_DIR=$O/logs \
  timeout -k 10 560 python -u -m pytest tests/test_libgeeps.py -m gpu -v -k "randomized" --timeout 250 \
  --timeout-method thread > $O/pytest_stress.log 2>&1
rc=$?; echo "stress rc=$rc $(tail -n 1 $O/pytest_stress.log)"; grep -E "FAILED" $O/pytest_stress.log | head -20
python scripts/ipc_audit.py $O/logs > $O/audit.json && python -c "import json; print(json.load(open('$O/audit.json'))['summary'])"
tar czf $O/logs.tgz -C $O logs && rm -rf $O/logs
exit $rc
