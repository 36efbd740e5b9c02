#!/bin/bash
# Round 4: where the first unplanned call with a new index spends its time
# (scripts/probes/first_call_breakdown.py: 8 M RowData rows, 3 fresh random
# indexes per op), host / event times, then the same under a kernel trace.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04dev11}; mkdir -p $O
timeout -k 10 200 python scripts/probes/first_call_breakdown.py > $O/first_call.json 2> $O/first_call.err; rc=$?
echo "first call rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/scripts/probes/first_call_breakdown.py > $O/first_call_prof.json 2> $O/first_call_prof.err; rc=$?
echo "prof rc=$rc"; exit $rc
