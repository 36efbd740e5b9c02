#!/bin/bash
# r05 dev1: the sticky unsound-map flag, stream-ordered plan retirement, the
# gloo-exchange + HIP-sum rehearsal of configs[2]; then smoke.
set -o pipefail
mkdir -p gpurun_out/r05dev1
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "unplanned" tests/test_rccl.py > gpurun_out/r05dev1/pytest.txt 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05dev1/smoke.txt 2>&1
rc=$?
tail -30 gpurun_out/r05dev1/pytest.txt
exit $rc
