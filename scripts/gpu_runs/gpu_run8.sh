#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
B=build/apps/geeps_clock_bench
timeout -k 10 200 $B 0 1 30100 $((1<<23)) 10 2 > gpurun_out/e2e_1p_8M.json 2> gpurun_out/e2e_1p_8M.err; rc=$?
echo "e2e 1p rc=$rc"; cat gpurun_out/e2e_1p_8M.json; tail -3 gpurun_out/e2e_1p_8M.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 $B 0 1 30100 $((1<<18)) 20 3 > gpurun_out/e2e_1p_256K.json 2>&1; echo "rc=$?"; cat gpurun_out/e2e_1p_256K.json
( timeout -k 10 300 $B 0 2 30200 $((1<<18)) 5 1 > gpurun_out/e2e_2p_p0.json 2>&1 & timeout -k 10 300 $B 1 2 30200 $((1<<18)) 5 1 > gpurun_out/e2e_2p_p1.json 2>&1; wait )
echo "2p done"; cat gpurun_out/e2e_2p_p0.json gpurun_out/e2e_2p_p1.json
exit 0
