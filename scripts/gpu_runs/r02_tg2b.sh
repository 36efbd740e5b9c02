#!/bin/bash
# Round 2: second fresh box for the bursts-of-2 headline: default bench and
# rocprofv3 kernel stats of the bench.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r02tg2b; mkdir -p $O
timeout -k 10 500 python bench.py > $O/bench_default.json 2> $O/bench_default.err; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/bench_default.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-host-inclusive --no-e2e > $O/prof_bench.json 2> $O/prof_bench.err; rc=$?
echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
