#!/bin/bash
# Round 2: bucket-sum plan-boundary fuzz (random bucket counts, in / out of
# place, sizes around the sweep / tile-major / mixed thresholds).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r02fz2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "boundaries_fuzz" -v --timeout 120 --timeout-method thread > $O/pytest_fuzz.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $O/pytest_fuzz.log)"; exit $rc
