#!/bin/bash
# Round 6: where the unplanned calls' first call with an index spends its time
# now (first_call_frac 0.59-0.66): the first-call probe
# under rocprofv3 kernel + HIP runtime traces (no counters).
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r06/dev7
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 $GRAFT_REPO_ROOT/scripts/probes/first_call_breakdown.py > $OUT/first_call.json 2> $OUT/first_call.err
rc=$?; echo "rc=$rc"; cat $OUT/first_call.json; exit $rc
