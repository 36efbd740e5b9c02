#!/bin/bash
# Round 3: kernel + memory-copy traces of the libgeeps clock bench with the
# direct oplog, 1 and 2 processes, for the per-clock timeline.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03trace}; mkdir -p $O
export TMPDIR=/tmp
for P in 1 2; do
  CLOCK_BENCH_PROF=$O/p$P timeout -k 10 300 python scripts/run_clock_bench.py $P 8388608 10 2 0 ipc $O/clock_p${P}.json > /dev/null 2>> $O/clock.err || exit 1
  python scripts/trace_timeline.py $O/p$P 30 > $O/timeline_p$P.txt 2>&1 || exit 1
done
cat $O/clock_p1.json $O/clock_p2.json; tail -40 $O/timeline_p2.txt
