#!/bin/bash
# r05 dev12: client.cpp split into client / client_viter / client_data /
# client_net (a move, no change of code): the libgeeps GPU suite.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r05dev12}; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_libgeeps.py tests/test_ipc.py -m gpu -v --timeout 175 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $O/pytest.log)"; grep FAILED $O/pytest.log | head; exit $rc
