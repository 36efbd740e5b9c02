#!/bin/bash
# Probe: register-phased scatter-add / fused init (one launch per chunk) vs the product, random + identity index.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r81; mkdir -p $O
timeout -k 10 300 ./build/tune/rowreg_tune 7 > $O/rowreg_a.txt 2> $O/a.err; rc=$?
echo "a rc=$rc"; cat $O/rowreg_a.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 ./build/tune/rowreg_tune 7 > $O/rowreg_b.txt 2> $O/b.err; rc=$?
echo "b rc=$rc"; cat $O/rowreg_b.txt; exit $rc
