#!/bin/bash
# Round 6: the rest of test_libgeeps.py's GPU cases (SSP, jitter, read-my-
# writes, configs[3] / configs[4], direct oplog / read, lagging readers, host
# tier, one process per GPU rehearsal, shuffled rows) with the TSan build of
# libgeeps and the sum app (scripts/build_tsan.sh), after tsan.sh's subset came
# back clean.  halt_on_error=0 and whole per-process logs: a report fails its
# test (exit 66) without hanging the peers, and is kept in full.
set -u
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r06/tsan_wide; mkdir -p $O
export PYTHONUNBUFFERED=1
export TSAN_OPTIONS="halt_on_error=0 second_deadlock_stack=1 report_signal_unsafe=0 history_size=4 suppressions=$GRAFT_REPO_ROOT/scripts/tsan.supp"
GEEPS_TEST_LOG_DIR=$O/logs GEEPS_SUM_APP=$GRAFT_REPO_ROOT/build/tsan/geeps_sum_app \
  timeout -k 10 1080 python -u -m pytest tests/test_libgeeps.py -m gpu -v \
  -k "not randomized and not two_processes and not ipc_failure and not peer_buckets and not peer_refresh" \
  --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "rc=$rc $(tail -n 1 $O/pytest.log)"; grep -E "FAILED" $O/pytest.log | head -20
grep -h "SUMMARY: ThreadSanitizer" $O/logs/*.log 2>/dev/null | sort | uniq -c
exit $rc
