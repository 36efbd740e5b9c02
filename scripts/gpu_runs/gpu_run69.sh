#!/bin/bash
# Row-op kernel rows-in-flight x blocks-per-CU sweep under the current cache policy.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r69; mkdir -p $O
timeout -k 10 300 ./build/tune/rowop_tune 8388608 7 > $O/rowop.txt 2> $O/rowop.err; rc=$?
echo "rc=$rc"; cat $O/rowop.txt; tail -n 3 $O/rowop.err; exit $rc
