#!/bin/bash
# Round 4: sums and row ops past the reference's int element range.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04dev14}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k "past_the_reference" --timeout 175 --timeout-method thread > $O/pytest_int_range.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $O/pytest_int_range.log)"; grep -E "FAILED|Error" $O/pytest_int_range.log | head -20; exit $rc
