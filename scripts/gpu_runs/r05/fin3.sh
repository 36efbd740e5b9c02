#!/bin/bash
# Round 5, the closing pass at the final code (after the host tier's fused
# init and one-copy runs): fin.sh (suite, smoke, bench, rocprofv3), then the
# 200-seed randomized libgeeps configurations.
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_runs/r05/fin.sh ${1:-r05fin3} || exit $?
bash scripts/gpu_runs/r05/campaign2.sh ${1:-r05fin3}
