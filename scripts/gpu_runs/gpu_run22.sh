#!/bin/bash
# Debug the SSP failures of the in-place refresh change: slack-2 4-process run
# and the AlexNet 8-process run, each process's stderr kept.
cd "$GRAFT_REPO_ROOT"
bash scripts/run_sum_app.sh gpurun_out/dbg/slack2 90 ipc 4 2048 12 2 1 0 int; rc=$?
echo "slack2 rc=$rc"; tail -n 30 gpurun_out/dbg/slack2/p*.err | cut -c1-300
bash scripts/run_sum_app.sh gpurun_out/dbg/alex 90 ipc 8 476292 4 1 1 0 int 273,1,2400,2,6912,3,5184,3,3456,2,294912,32,131072,32,32000,8; rc2=$?
echo "alex rc=$rc2"; tail -n 12 gpurun_out/dbg/alex/p*.err | cut -c1-300
exit 0
