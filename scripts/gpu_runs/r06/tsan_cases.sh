#!/bin/bash
# Round 6: the three cases ThreadSanitizer stopped in (tsan.sh), again with
# every process's whole output kept (GEEPS_TEST_LOG_DIR) and without
# halt_on_error, so each report is read in full and the peers do not hang.
set -u
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r06/tsan_cases; mkdir -p $O
export PYTHONUNBUFFERED=1
export TSAN_OPTIONS="halt_on_error=0 second_deadlock_stack=1 report_signal_unsafe=0 history_size=4 suppressions=$GRAFT_REPO_ROOT/scripts/tsan.supp"
GEEPS_TEST_LOG_DIR=$O/logs GEEPS_SUM_APP=$GRAFT_REPO_ROOT/build/tsan/geeps_sum_app GEEPS_STRESS_CASES=20 \
  timeout -k 10 500 python -u -m pytest tests/test_libgeeps.py -m gpu -v \
  -k "test_ipc_failure_costs_a_resend_not_the_job and tag-3-1-extra1 or test_randomized_configurations and (1] or 16])" \
  --timeout 250 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "rc=$rc $(tail -n 1 $O/pytest.log)"
grep -h "SUMMARY: ThreadSanitizer" $O/logs/*.log | sort | uniq -c
exit $rc
