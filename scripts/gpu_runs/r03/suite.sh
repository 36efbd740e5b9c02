#!/bin/bash
# Round 3: GPU suite (verbose) + smoke, no bench.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03suite}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 175 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $O/pytest_gpu.log)"; grep -E "FAILED|Error|passed,|failed," $O/pytest_gpu.log | head -20
grep -A16 "geeps parity summary" $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; rc2=$?
echo "smoke rc=$rc2"; tail -2 $O/smoke.txt; exit $rc2
