#!/bin/bash
# Row-op stream cache policy probe (nt on x loads / y loads / y stores).
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r57; mkdir -p $O
timeout -k 10 300 ./build/tune/rownt_tune 7 > $O/rownt.txt 2> $O/rownt.err; rc=$?
echo "rc=$rc"; cat $O/rownt.txt; tail -n 3 $O/rownt.err; exit $rc
