#!/bin/bash
# Round 4: the unplanned-call parity tests (stats counters, repeated
# destinations) and the ABI / C99 checks after ABI 12.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04dev13}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_abi.py -m gpu -v -k "unplanned or c_abi or abi" --timeout 175 --timeout-method thread > $O/pytest_unplanned.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $O/pytest_unplanned.log)"; grep -E "FAILED|Error" $O/pytest_unplanned.log | head -20; exit $rc
