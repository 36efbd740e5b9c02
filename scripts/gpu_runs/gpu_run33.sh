#!/bin/bash
# Full GPU suite + smoke + default bench after the zero-copy refresh and stream changes.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r33; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc $(grep -o '"frac": [0-9.]*' $O/bench.json | head -1) $(grep -o '"avg_kernel_ms": [0-9.]*' $O/bench.json | head -1)"; exit $rc
