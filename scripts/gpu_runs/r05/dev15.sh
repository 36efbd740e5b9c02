#!/bin/bash
# r05 dev15: host-tier ops whose rows are one run of host rows: one copy for Read and (fused) Update; as dev14:
# the persistent host worker pool: host-tier tests incl. the multi-piece ops,
# then the timer breakdown (shared oplogs, in-frame rows).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r05dev15}; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_host_rows.py tests/test_hostshare.py tests/test_libgeeps.py tests/test_gpu_parity.py -m gpu -v -k "host or mm_level or ipc_failure or page_locked or c_abi" --timeout 150 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $O/pytest.log)"; grep FAILED $O/pytest.log | head; [ $rc -eq 0 ] || exit $rc
for share in 1 0; do
timeout -k 10 200 python -c "
import json, sys
sys.path.insert(0, 'scripts')
import run_clock_bench as m
r = m.run(2, 476292, 10, 5, 0, 'ipc', timeout=120, extra_env={'CLOCK_BENCH_HOST_TIER_FRAC': '0.5', 'GEEPS_HOST_SHARE': '$share'})
print(json.dumps({'ms_per_clock': r['ms_per_clock'], 'read_ok': r['read_ok'], 'nr_host_shared': r['nr_host_shared'],
                  'client': [s['client'] for s in r['stats']], 'servers': [s['servers'] for s in r['stats']]}))
" > $O/host_tier_share$share.json 2> $O/host_tier_share$share.err; rc=$?
echo "share=$share rc=$rc $(head -c 120 $O/host_tier_share$share.json)"; [ $rc -eq 0 ] || exit $rc
done
