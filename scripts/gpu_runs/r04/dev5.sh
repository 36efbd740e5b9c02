#!/bin/bash
# Round 4, fifth GPU pass: IPC priming (primed vs late, 10 runs each) and the
# first-call breakdown of the unplanned scatter-add / init (kernel trace).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04dev5}; mkdir -p $O
timeout -k 10 500 python -u scripts/probes/ipc_probe.py late primed late primed late primed late primed late primed late primed late primed late primed late primed late primed > $O/ipc_primed.jsonl 2> $O/ipc_primed.err; echo "ipc primed rc=$?"
timeout -k 10 200 python scripts/probes/first_call_breakdown.py > $O/first_call.json 2> $O/first_call.err; echo "first call rc=$?"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/scripts/probes/first_call_breakdown.py > $O/first_call_prof.json 2> $O/first_call_prof.err; echo "prof rc=$?"
