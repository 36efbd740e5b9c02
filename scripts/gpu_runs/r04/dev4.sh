#!/bin/bash
# Round 4, fourth GPU pass: does a throwaway first allocation avoid the IPC
# failures of a process's first buffer (warm vs late, 8 runs each); the
# unplanned-call tests with the inverse plan; the client row-op legs.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04dev4}; mkdir -p $O
timeout -k 10 500 python -u scripts/probes/ipc_probe.py late warm late warm late warm late warm late warm late warm late warm late warm > $O/ipc_warm.jsonl 2> $O/ipc_warm.err; echo "ipc warm rc=$?"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 175 --timeout-method thread \
  -k "unplanned or golden or scatter_init or full_size_scatter or rowop" > $O/pytest_sel.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $O/pytest_sel.log)"; grep -E "FAILED|Error" $O/pytest_sel.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-inclusive --no-config2 --no-e2e \
  --no-per-rank --no-pmc --no-separate-alloc --no-hbm-probe > $O/bench_rowops.json 2> $O/bench_rowops.err; rc=$?
echo "bench rowops rc=$rc"; exit $rc
