#!/bin/bash
# r05 dev4: the host tier with pinned buffers and threaded host row ops: its
# tests, then the libgeeps clock leg (the host-tier run among them).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r05dev4}; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_libgeeps.py -m gpu -v -x --timeout 175 --timeout-method thread -k "host_tier or mm_level or ipc_failure" > $O/pytest_host_tier.log 2>&1; rc=$?
echo "host tier rc=$rc $(tail -n 1 $O/pytest_host_tier.log)"; grep -E "FAILED|Error" $O/pytest_host_tier.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -c "import json, bench; print(json.dumps(bench.libgeeps_leg(1 << 20, 1024)))" > $O/libgeeps_leg.json 2> $O/libgeeps_leg.err; rc=$?
echo "leg rc=$rc"; cat $O/libgeeps_leg.json; exit $rc
