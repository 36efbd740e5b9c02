#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_libgeeps.py -m gpu -q -x --durations=8 > gpurun_out/pytest11.log 2>&1; rc=$?
echo "libgeeps pytest rc=$rc"; tail -25 gpurun_out/pytest11.log
if [ $rc -ne 0 ]; then exit $rc; fi
B=$GRAFT_REPO_ROOT/build/apps/geeps_clock_bench
for T in ipc tcp; do
  ( GEEPS_TRANSPORT=$T timeout -k 10 300 $B 0 2 30200 $((1<<18)) 10 2 > gpurun_out/e2e11_${T}_p0.json 2>gpurun_out/e2e11_${T}_p0.err & GEEPS_TRANSPORT=$T timeout -k 10 300 $B 1 2 30200 $((1<<18)) 10 2 > gpurun_out/e2e11_${T}_p1.json 2>gpurun_out/e2e11_${T}_p1.err; wait )
  echo "e2e 2p $T"; cat gpurun_out/e2e11_${T}_p0.json gpurun_out/e2e11_${T}_p1.json
done
exit 0
