#!/bin/bash
# Evidence set for the phase-separated sum: full GPU suite, smoke, default bench,
# headline-only rocprofv3 kernel-trace summary, FETCH_SIZE / WRITE_SIZE passes.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r41; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 $O/pytest_gpu.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err; rc=$?
echo "bench rc=$rc"; cat $O/bench_default.json; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu-baseline --no-host-inclusive --no-rowops --no-hbm-probe"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $O/prof_bench.json 2> $O/prof_bench.err; rc=$?
echo "rocprof rc=$rc"; cat $O/prof_bench.json; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS --steps 2 --warmup 1 > $O/pmc_fetch.log 2>&1; rc=$?
echo "pmc fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS --steps 2 --warmup 1 > $O/pmc_write.log 2>&1; rc=$?
echo "pmc write rc=$rc"; exit $rc
