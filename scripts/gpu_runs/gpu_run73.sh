#!/bin/bash
# Row-op index-map forms (per-lane / LDS-staged map / wave shfl) A/B under the current cache policy.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r73; mkdir -p $O
timeout -k 10 400 ./build/tune/rowmap_tune 5 > $O/rowmap.txt 2> $O/rowmap.err; rc=$?
echo "rc=$rc"; cat $O/rowmap.txt; tail -n 3 $O/rowmap.err; exit $rc
