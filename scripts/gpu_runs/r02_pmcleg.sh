#!/bin/bash
# Round 2: bench.py with the in-run PMC traffic passes (rocprofv3 child
# processes), then the same bench under rocprofv3 --kernel-trace --stats
# (which must skip the PMC passes).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r02pmcleg; mkdir -p $O
start=$(date +%s)
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err; rc=$?
echo "bench rc=$rc wall=$(( $(date +%s) - start ))s"; [ $rc -eq 0 ] || { tail -20 $O/bench_default.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-host-inclusive --no-e2e > $O/prof_bench.json 2> $O/prof_bench.err; rc=$?
echo "rocprof rc=$rc"; grep -c "PMC traffic passes" $O/prof_bench.err; exit $rc
