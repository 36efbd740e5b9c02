#!/bin/bash
# Round 6: the library split (gp_kernels.hpp shared by gp_reduce.hip and
# gp_unplanned.hip; no kernel's code changed): the GPU suite, smoke, and the
# default bench line, to confirm parity and rates are those of dev1 / dev2.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r06/dev6
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -24 $OUT/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
rc=$?; echo "bench rc=$rc"; exit $rc
