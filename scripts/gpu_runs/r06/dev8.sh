#!/bin/bash
# Round 6: bench.py's N > 1 libgeeps leg, rehearsed on one GPU (2 processes;
# both cross-GPU paths forced), and the new verdict scalars computed from its
# real output (bench.multi_gpu_verdict).  On one GPU staging is pure extra HBM
# traffic, so in place is expected to win here; only an 8-GPU node decides.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r06/dev8
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -c "
import json, bench
r = bench.libgeeps_multi_gpu_leg(2, 1 << 20, 1024)
print(json.dumps({'leg': r, 'verdict': bench.multi_gpu_verdict(r)}))
" > $OUT/multi_leg.json 2> $OUT/multi_leg.err
rc=$?; echo "rc=$rc"; cat $OUT/multi_leg.json; exit $rc
