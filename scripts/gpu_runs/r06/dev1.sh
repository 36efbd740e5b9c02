#!/bin/bash
# Round 6, first GPU pass: the whole -m gpu suite after the gp_runtime.hip split
# (IPC diagnostics, ABI 16) with the 8-rank configs[2]-shape rehearsal, then
# round 5's two failing randomized seeds (256, 285: GEEPS_TEST_IPC_FAULT=refuse
# at P = 4) ONCE, with every process's IPC audit (GEEPS_IPC_LOG) kept whole.
# A step that ends in a fault, abort, timeout or kill ends the script.
set -u
OUT=gpurun_out/r06/dev1
mkdir -p $OUT
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # pass, or ordinary test failures

timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $OUT/pytest_gpu.txt 2>&1
rc=$?; echo "pytest -m gpu rc=$rc"; tail -30 $OUT/pytest_gpu.txt
ok $rc || exit $rc

GEEPS_STRESS_CASES=300 GEEPS_IPC_LOG=1 GEEPS_TEST_LOG_DIR=$OUT/seeds \
  timeout -k 10 600 python -u -m pytest -v --timeout 240 --timeout-method thread \
  "tests/test_libgeeps.py::test_randomized_configurations[256]" \
  "tests/test_libgeeps.py::test_randomized_configurations[285]" > $OUT/seeds.txt 2>&1
rc=$?; echo "seeds rc=$rc"; tail -20 $OUT/seeds.txt
exit $rc
