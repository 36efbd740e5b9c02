#!/bin/bash
# Round 3 probe 6: the unplanned call's first-call cost, with a HIP API trace.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03first}; mkdir -p $O
timeout -k 10 200 python scripts/probes/first_call.py > $O/plain.txt 2>&1 || exit 1
cat $O/plain.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/scripts/probes/first_call.py > $O/traced.txt 2>&1; rc=$?
echo "rocprof rc=$rc"; cat $O/traced.txt | tail -12; exit $rc
