#!/bin/bash
# Round 4, sixth GPU pass (no probes): the whole GPU suite (tagged IPC
# buffers, inverse plan from the stream-ordered pool), then the client row-op
# legs.  Every step under its own time limit; stop at the first failure.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04dev6}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 175 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $O/pytest_gpu.log)"; grep -E "FAILED" $O/pytest_gpu.log | head -20
grep -A19 "geeps parity summary" $O/pytest_gpu.log | tail -19
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-inclusive --no-config2 --no-e2e \
  --no-per-rank --no-pmc --no-separate-alloc --no-hbm-probe > $O/bench_rowops.json 2> $O/bench_rowops.err; rc=$?
echo "bench rowops rc=$rc"; exit $rc
