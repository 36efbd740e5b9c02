#!/bin/bash
# Round 6: bench.py at N = 1 after the library split (gp_runtime.hip) -- the
# suite ran in dev1, the bench had not -- with rocprofv3 kernel stats of the
# same command, so the round's profile summary comes from its own code.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r06/dev2
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 420 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
rc=$?; echo "bench rc=$rc"; tail -c 600 $OUT/bench_default.json; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-host-inclusive --no-e2e \
  > $OUT/prof_bench.json 2> $OUT/prof_bench.err
rc=$?; echo "rocprof rc=$rc"; exit $rc
