#!/bin/bash
# Round 2: plans with dense runs again -- parity, the allocation sweep, PMC of
# the planned identity legs (now the phased 1-bucket sum / its ZIN form).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r02k; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "row_plan or scatter_init or bucket" -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $O/pytest.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/tune/rowop_alloc.py 10 > $O/rowop_alloc3.txt 2>&1; rc=$?
echo "alloc rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
B=$GRAFT_REPO_ROOT/bench.py
BASE="--no-cpu-baseline --no-host-inclusive --no-hbm-probe --no-config2 --steps 1 --warmup 0"
for leg in scatter_add_planned scatter_init_planned; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_${leg}_identity_$c -o run -- python3 $B $BASE --rowops-only $leg --rowops-index identity > $O/pmc_${leg}_$c.log 2>&1; rc=$?
    echo "$leg $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
