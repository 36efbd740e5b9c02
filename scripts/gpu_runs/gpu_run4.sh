#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 420 python -m pytest tests/test_libgeeps.py -m gpu -q -x > gpurun_out/pytest_libgeeps.log 2>&1; rc=$?
echo "libgeeps pytest rc=$rc"; tail -30 gpurun_out/pytest_libgeeps.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu4.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu4.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 20 --warmup 3 > gpurun_out/bench4.json 2> gpurun_out/bench4.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench4.json
exit $rc
