#!/bin/bash
# Probe: bucket-major read phase (one stream at a time, LDS/register accumulate) vs production, 8 and 2 buckets, 3 arenas.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r84; mkdir -p $O
timeout -k 10 400 ./build/tune/bmaj_tune 7 3 > $O/bmaj_a.txt 2> $O/a.err; rc=$?
echo "a rc=$rc"; cat $O/bmaj_a.txt; exit $rc
