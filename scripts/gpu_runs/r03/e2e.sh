#!/bin/bash
# Round 3: direct oplog -- libgeeps GPU tests, then the clock bench with the
# direct oplog on (default) and off (GEEPS_DIRECT_OPLOG=0), 1 and 2 workers.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03e2e}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_libgeeps.py -m gpu -v --timeout 175 --timeout-method thread > $O/pytest_libgeeps.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $O/pytest_libgeeps.log)"; grep -E "FAILED|passed,|failed," $O/pytest_libgeeps.log | head -20
[ $rc -eq 0 ] || exit $rc
for P in 1 2; do
  timeout -k 10 200 python scripts/run_clock_bench.py $P 8388608 10 2 0 ipc $O/clock_p${P}_direct.json > /dev/null 2>> $O/clock.err || exit 1
  GEEPS_DIRECT_OPLOG=0 timeout -k 10 200 python scripts/run_clock_bench.py $P 8388608 10 2 0 ipc $O/clock_p${P}_copy.json > /dev/null 2>> $O/clock.err || exit 1
done
for f in $O/clock_*.json; do echo "$(basename $f) $(cat $f)"; done
