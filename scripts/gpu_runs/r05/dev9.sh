#!/bin/bash
# r05 dev9: host tier with the threaded oplog zero: its tests, the C99 ABI
# check (host row ops now in it), then the timer breakdown again.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r05dev9}; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_libgeeps.py tests/test_gpu_parity.py -m gpu -v -k "host_tier or mm_level or c_abi" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $O/pytest.log)"; grep FAILED $O/pytest.log | head; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_runs/r05/dev8.sh ${1:-r05dev9}
