#!/bin/bash
# The driver's round-end commands on a fresh box: GPU suite, smoke, default bench.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r72; mkdir -p $O
timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > $O/pytest_gpu.log 2>&1; rc=$?
echo "gpu suite rc=$rc $(tail -n 1 $O/pytest_gpu.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc $(tail -n 1 $O/smoke.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc $(grep -o '"avg_kernel_ms": [0-9.]*' $O/bench.json | head -1) $(grep -o '"frac": [0-9.]*' $O/bench.json | tr '\n' ' ')"; exit $rc
