#!/bin/bash
# Round 3: plan cache built on the second sighting -- the unplanned / plan-cache
# GPU tests, the first-call probe, and the bench's row-op legs.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03cache}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k "unplanned or rowop or scatter or gather or golden" --timeout 175 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $O/pytest.log)"; grep FAILED $O/pytest.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/probes/first_call.py > $O/first_call.txt 2>&1 || exit 1
cat $O/first_call.txt
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-inclusive --no-config2 --no-e2e --no-per-rank --no-pmc --no-separate-alloc > $O/bench_rowops.json 2> $O/bench_rowops.err; rc=$?
echo "bench rc=$rc"; exit $rc
