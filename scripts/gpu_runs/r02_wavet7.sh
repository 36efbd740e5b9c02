#!/bin/bash
# Round 2: rows in flight / blocks per CU for the wave-map row kernel on a row
# plan's random residual (scripts/tune/wave_tune.hip).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r02wavet; mkdir -p $O
timeout -k 10 400 ./build/tune/wave_tune 9 > $O/wave_tune7.txt 2> $O/wave_tune7.err; rc=$?
echo "wave_tune rc=$rc"; cat $O/wave_tune7.txt; exit $rc
