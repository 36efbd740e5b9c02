#!/bin/bash
# Round 2: the plain-C99 C-ABI consumer on the GPU (tests/apps/c_abi_check.c).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r02cabi; mkdir -p $O
timeout -k 10 120 ./build/tests/c_abi_check > $O/c_abi_check.txt 2>&1; rc=$?
echo "c_abi_check rc=$rc"; cat $O/c_abi_check.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k c_abi -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_cabi.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $O/pytest_cabi.log)"; [ $rc -eq 0 ] || exit $rc
