#!/bin/bash
# r05 dev6: host-tier pushes over IPC, randomized configs with host tiers and
# IPC faults: the libgeeps suite (40 random cases), then the clock legs.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r05dev6}; mkdir -p $O
export PYTHONUNBUFFERED=1
GEEPS_STRESS_CASES=40 timeout -k 10 800 python -u -m pytest tests/test_libgeeps.py -m gpu -v --timeout 175 --timeout-method thread > $O/pytest_libgeeps.log 2>&1; rc=$?
echo "libgeeps rc=$rc $(tail -n 1 $O/pytest_libgeeps.log)"; grep -E "FAILED" $O/pytest_libgeeps.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -c "import json, bench; print(json.dumps(bench.libgeeps_leg(1 << 20, 1024)))" > $O/libgeeps_leg.json 2> $O/libgeeps_leg.err; rc=$?
echo "leg rc=$rc"; python -c "import json; d=json.load(open('$O/libgeeps_leg.json')); print({k: (v.get('ms_per_clock'), v.get('read_ok')) for k, v in d.items() if isinstance(v, dict)})"; exit $rc
