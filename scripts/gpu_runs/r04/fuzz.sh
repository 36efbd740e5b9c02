#!/bin/bash
# Round 4: a wider parity fuzz campaign (row plans, unplanned calls with the
# plan cache, bucket-sum plan boundaries), bit for bit against the oracle.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04fuzz}; mkdir -p $O
GEEPS_FUZZ_CASES=${2:-200} timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "fuzz" --timeout 175 --timeout-method thread > $O/pytest_fuzz.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $O/pytest_fuzz.log)"; grep -E "FAILED" $O/pytest_fuzz.log | head; grep -A6 "parity summary" $O/pytest_fuzz.log; exit $rc
