#!/bin/bash
# Round 6: multi-chunk sweep launches (scripts/tune/r6_multichunk_tune.hip):
# P chunks per launch vs one, at 2 buckets (configs[1]) and 8 (the headline),
# bit-checked against production, interleaved rounds, under rocprofv3 kernel
# stats (register / scratch use per variant in the trace).
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r06/dev3
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  $GRAFT_REPO_ROOT/build/r6probe/r6_multichunk_tune 7 > $OUT/multichunk.txt 2> $OUT/multichunk.err
rc=$?; echo "rc=$rc"; cat $OUT/multichunk.txt; exit $rc
