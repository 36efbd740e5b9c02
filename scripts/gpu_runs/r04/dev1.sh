#!/bin/bash
# Round 4, first GPU pass: the IPC probe, the changed parity / libgeeps tests,
# the client row-op legs (steady-state unplanned calls), and the one-GPU
# rehearsal of bench.py's one-process-per-GPU libgeeps leg.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04dev1}; mkdir -p $O
timeout -k 10 330 python -u scripts/probes/ipc_probe.py > $O/ipc_probe.jsonl 2> $O/ipc_probe.err; echo "ipc probe rc=$?"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_libgeeps.py -m gpu -v --timeout 175 --timeout-method thread \
  -k "unplanned or direct_read or capacity or shuffled or one_process or direct_oplog or peer" > $O/pytest_sel.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $O/pytest_sel.log)"; grep -E "FAILED|Error" $O/pytest_sel.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-inclusive --no-config2 --no-e2e \
  --no-per-rank --no-pmc --no-separate-alloc --no-hbm-probe > $O/bench_rowops.json 2> $O/bench_rowops.err; rc=$?
echo "bench rowops rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -c "
import json, bench
r = bench.libgeeps_multi_gpu_leg(2, 1 << 20, 1024, gpus_seen=1)
print(json.dumps(r))
r = bench.libgeeps_multi_gpu_leg(8, 1 << 20, 1024, gpus_seen=1, tables=('alexnet',))
print(json.dumps(r))
" > $O/multi_rehearsal.jsonl 2> $O/multi_rehearsal.err; rc=$?
echo "multi rehearsal rc=$rc"; exit $rc
