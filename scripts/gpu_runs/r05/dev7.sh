#!/bin/bash
# r05 dev7: first calls of the unplanned row ops after the plan-retirement
# change (entries whose calls are done are freed at once again): the
# unplanned tests, then the client row-op leg.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r05dev7}; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k "unplanned" --timeout 120 --timeout-method thread > $O/pytest_unplanned.log 2>&1; rc=$?
echo "unplanned rc=$rc $(tail -n 1 $O/pytest_unplanned.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "
import json, torch, bench
r = bench.rowops_leg(1 << 20, 1024, torch.device('cuda', 0))
print(json.dumps(r))" > $O/rowops.json 2> $O/rowops.err; rc=$?
echo "rowops rc=$rc"; python -c "
import json; r = json.load(open('$O/rowops.json'))
for kind in ('random', 'identity'):
    for leg, v in r[kind].items():
        if isinstance(v, dict) and 'frac' in v: print(kind, leg, v.get('avg_ms'), v['frac'], v.get('first_call_ms'))"; exit $rc
