#!/bin/bash
# Round 6: libgeeps under ThreadSanitizer (host code only: scripts/build_tsan.sh;
# the HIP runtime and kernels are not instrumented) after this round's
# libgeeps changes (parked IPC mappings per client reader, kept mis-mappings):
# the two-process cases, staged peers, the IPC-failure recovery (NACK /
# resend, replaced oplog buffers: the parking path) and 20 randomized seeds.
# First, one short run to see the sanitizer starts beside the HIP runtime.
set -u
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r06/tsan; mkdir -p $O
export PYTHONUNBUFFERED=1
export TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1 report_signal_unsafe=0 suppressions=$GRAFT_REPO_ROOT/scripts/tsan.supp"
APP=$GRAFT_REPO_ROOT/build/tsan/geeps_sum_app
GEEPS_SUM_APP=$APP timeout -k 10 240 python -u -m pytest tests/test_libgeeps.py -m gpu -v -x \
  -k "test_two_processes_loopback_bsp" --timeout 200 --timeout-method thread > $O/pytest_first.log 2>&1
rc=$?; echo "first rc=$rc $(tail -n 1 $O/pytest_first.log)"; grep -m5 -E "ThreadSanitizer|FAILED" $O/pytest_first.log
[ $rc -eq 0 ] || exit $rc
GEEPS_SUM_APP=$APP GEEPS_STRESS_CASES=20 timeout -k 10 800 python -u -m pytest tests/test_libgeeps.py -m gpu -v \
  -k "two_processes or ipc_failure or peer_buckets or peer_refresh or randomized" --timeout 250 \
  --timeout-method thread > $O/pytest_tsan.log 2>&1
rc=$?; echo "tsan rc=$rc $(tail -n 1 $O/pytest_tsan.log)"; grep -E "FAILED" $O/pytest_tsan.log | head -20
grep -m3 -A20 "WARNING: ThreadSanitizer" $O/pytest_tsan.log | head -60
exit $rc
