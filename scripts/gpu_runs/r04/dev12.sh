#!/bin/bash
# Round 4: the GPU suite, the client row-op legs, then the first-call
# breakdown under a kernel trace (after the once-per-launch flag writes and
# the block-reduced inverse-map count).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04dev12}
bash scripts/gpu_runs/r04/dev6.sh ${1:-r04dev12} || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/scripts/probes/first_call_breakdown.py > $O/first_call_prof.json 2> $O/first_call_prof.err; rc=$?
echo "prof rc=$rc"; exit $rc
