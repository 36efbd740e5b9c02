#!/bin/bash
# Round 6: one sweep chunk per launch at other chunk sizes (register tiles),
# at 2 buckets (configs[1]) and 8 (the headline), bit-checked against
# production, interleaved rounds, under rocprofv3 kernel stats
# (scripts/tune/r6_multichunk_tune.hip built with -DR6_CHUNK_SIZES).
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r06/dev4
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  $GRAFT_REPO_ROOT/build/r6probe/r6_chunksize_tune 7 > $OUT/chunksize.txt 2> $OUT/chunksize.err
rc=$?; echo "rc=$rc"; cat $OUT/chunksize.txt; exit $rc
