#!/bin/bash
# Round 3: scan v3 (readlane density tests) timed in the probe, then the
# unplanned / plan-cache parity tests.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r03scan2; mkdir -p $O
timeout -k 10 300 ./build/probe/r3_row_tune2 5 > $O/r3_row_tune2d.txt 2> $O/r3_row_tune2d.err; rc=$?
echo "probe rc=$rc"; head -12 $O/r3_row_tune2d.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 175 --timeout-method thread -k "unplanned or golden or rowop" > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $O/pytest.log)"; grep FAILED $O/pytest.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 ./build/probe/r3_wave_tune 5 > $O/r3_wave_tune.txt 2> $O/r3_wave_tune.err; rc=$?
echo "wave probe rc=$rc"; cat $O/r3_wave_tune.txt; exit $rc
