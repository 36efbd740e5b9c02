#!/bin/bash
# Round 4: loopback-TCP clock A/B on one box: the refresh's rows streamed
# into HBM during the receive (GEEPS_STREAM_RECV=1) or landed whole first (0),
# three runs each, interleaved.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04dev24}; mkdir -p $O
for i in 1 2 3; do
  for v in 1 0; do
    GEEPS_STREAM_RECV=$v timeout -k 10 120 python scripts/run_clock_bench.py 2 476292 10 2 0 tcp > $O/tcp_${v}_${i}.json 2> $O/tcp_err_${v}_${i}.txt || exit 1
    echo "stream=$v run=$i $(python -c "import json,sys; print(json.load(open('$O/tcp_${v}_${i}.json'))['ms_per_clock_max'])")"
  done
done
