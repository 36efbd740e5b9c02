#!/bin/bash
# Phased sum over arenas with 0 / 4 KiB / 16 KiB / 68 KiB / 1 MiB+4 KiB between buffers; two processes.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r70; mkdir -p $O
PHASE_TUNE_PADS=1 timeout -k 10 300 ./build/tune/phase_tune 5 5 > $O/phase_pads_a.txt 2> $O/phase_pads_a.err; rc=$?
echo "a rc=$rc"; [ $rc -eq 0 ] || exit $rc
PHASE_TUNE_PADS=1 timeout -k 10 300 ./build/tune/phase_tune 5 5 > $O/phase_pads_b.txt 2> $O/phase_pads_b.err; rc=$?
echo "b rc=$rc"; cat $O/phase_pads_a.txt $O/phase_pads_b.txt | grep -v mismatch; exit $rc
