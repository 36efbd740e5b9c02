#!/bin/bash
# Round 4, second GPU pass: IPC probe (mappings kept open, concurrent opens /
# exports of fragments sharing a block), the unplanned-call parity tests, the
# client row-op legs (compact check + one select launch).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04dev2}; mkdir -p $O
timeout -k 10 400 python -u scripts/probes/ipc_probe.py keep mt_open mt_open mt_open mt_open mt_open mt_open mt_export mt_export mt_export > $O/ipc_probe.jsonl 2> $O/ipc_probe.err; echo "ipc probe rc=$?"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 175 --timeout-method thread \
  -k "unplanned or golden or scatter_init or full_size_scatter" > $O/pytest_sel.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $O/pytest_sel.log)"; grep -E "FAILED|Error" $O/pytest_sel.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-inclusive --no-config2 --no-e2e \
  --no-per-rank --no-pmc --no-separate-alloc --no-hbm-probe > $O/bench_rowops.json 2> $O/bench_rowops.err; rc=$?
echo "bench rowops rc=$rc"; exit $rc
