#!/bin/bash
# Round 4: the multi-GPU bench leg's code at 8 processes on one GPU (AlexNet
# table only; staging forced, so 7 peer readers each land refreshes in their
# own buffer and the servers copy on 8 streams), as the driver's N = 8 run will.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04dev28}; mkdir -p $O
timeout -k 10 300 python -c "import json, bench; print(json.dumps(bench.libgeeps_multi_gpu_leg(8, 1 << 20, 1024, gpus_seen=1, tables=('alexnet',))))" > $O/multi8.json 2> $O/multi8.err; rc=$?
echo "rc=$rc"; cat $O/multi8.json; exit $rc
