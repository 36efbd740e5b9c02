#!/bin/bash
# Full-size parity: every element of the 36-GiB 8-way sum and the 8M-row scatter-add vs torch.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r65; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k full_size --timeout 300 --timeout-method thread > $O/pytest_full.log 2>&1; rc=$?
echo "full-size rc=$rc $(tail -n 1 $O/pytest_full.log)"; exit $rc
