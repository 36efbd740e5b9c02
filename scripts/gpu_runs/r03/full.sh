#!/bin/bash
# Round 3: GPU suite (verbose: each test's name is in the log as it starts),
# smoke, default bench.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03full}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 175 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $O/pytest_gpu.log)"; grep -E "FAILED|passed,|failed," $O/pytest_gpu.log | head -20
grep -A14 "geeps parity summary" $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; rc2=$?
echo "smoke rc=$rc2"; cat $O/smoke.txt | tail -2; [ $rc2 -eq 0 ] || exit $rc2
timeout -k 10 500 python bench.py > $O/bench_default.json 2> $O/bench_default.err; rc3=$?
echo "bench rc=$rc3"; exit $rc3
