#!/bin/bash
# Probe: bucket-major read phase, register-tile and burst sweep at 8, 4, 2, 1 buckets vs production, 3 arenas.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r85; mkdir -p $O
timeout -k 10 400 ./build/tune/bmaj_tune 7 3 > $O/bmaj_b.txt 2> $O/a.err; rc=$?
echo "a rc=$rc"; cat $O/bmaj_b.txt; exit $rc
