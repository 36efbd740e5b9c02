#!/bin/bash
# Round 2: fuzzed row / gather plans against the oracle.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r02f; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "fuzz or plan" -x -v --timeout 300 --timeout-method thread > $O/pytest_fuzz.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $O/pytest_fuzz.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest_fuzz.log | head -20; exit $rc; }
