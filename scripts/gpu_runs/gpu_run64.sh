#!/bin/bash
# FETCH/WRITE passes over the bench's row-op leg after the cache-policy change.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r64; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu-baseline --no-host-inclusive --no-hbm-probe --steps 1 --warmup 0"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $O/pmc_fetch.log 2>&1; rc=$?
echo "pmc fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $O/pmc_write.log 2>&1; rc=$?
echo "pmc write rc=$rc"; exit $rc
