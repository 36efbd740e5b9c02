#!/bin/bash
# Round-1b evidence set on the final kernels: default bench line, headline-only
# rocprofv3 kernel-trace summary, FETCH_SIZE / WRITE_SIZE passes (own runs), and
# the 2-client (BASELINE configs[1]) reduction.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r26
mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err; rc=$?
echo "bench rc=$rc"; cat $O/bench_default.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --clients 2 --no-cpu-baseline --no-host-inclusive --no-rowops > $O/bench_2clients.json 2> $O/bench_2clients.err; rc=$?
echo "bench2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu-baseline --no-host-inclusive --no-rowops --no-hbm-probe"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $O/prof_bench.json 2> $O/prof_bench.err; rc=$?
echo "rocprof rc=$rc"; cat $O/prof_bench.json; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS --steps 3 --warmup 1 > $O/pmc_fetch.log 2>&1; rc=$?
echo "pmc fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS --steps 3 --warmup 1 > $O/pmc_write.log 2>&1; rc=$?
echo "pmc write rc=$rc"; exit $rc
