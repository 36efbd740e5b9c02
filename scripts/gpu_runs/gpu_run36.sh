#!/bin/bash
# Debug the jittered slack-3 IPC hang: each process's stderr kept.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r36; mkdir -p $O
GEEPS_TEST_JITTER_US=3000 bash scripts/run_sum_app.sh $O/s3j 60 ipc 4 1500 25 3 2 0 int; rc=$?
echo "s3j rc=$rc"; for f in $O/s3j/p*.err; do echo "== $f"; tail -n 8 $f | cut -c1-300; done
exit $rc
