#!/bin/bash
# Round 4, third GPU pass: IPC export/import of 1-MB fragments vs whole 2-MiB
# allocations (5 runs x 256 buffers each), then the whole GPU suite with
# libgeeps' IPC buffers allocated whole (gp_malloc_device_shared).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04dev3}; mkdir -p $O
timeout -k 10 500 python -u scripts/probes/ipc_probe.py stress_frag stress_whole stress_frag stress_whole stress_frag stress_whole stress_frag stress_whole stress_frag stress_whole > $O/ipc_stress.jsonl 2> $O/ipc_stress.err; echo "ipc stress rc=$?"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 175 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $O/pytest_gpu.log)"; grep -E "FAILED" $O/pytest_gpu.log | head -20
grep -A18 "geeps parity summary" $O/pytest_gpu.log | tail -18
exit $rc
