#!/bin/bash
# Round 3: direct read -- the direct-read tests first, then every libgeeps GPU
# test, then the 1-worker clock bench with direct reads on and off.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03dread}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_libgeeps.py -m gpu -v -s -k direct_read --timeout 175 --timeout-method thread > $O/pytest_dread.log 2>&1; rc=$?
echo "pytest dread rc=$rc $(tail -n 1 $O/pytest_dread.log)"; grep -E "FAILED|direct reads:" $O/pytest_dread.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests/test_libgeeps.py -m gpu -v --timeout 175 --timeout-method thread > $O/pytest_libgeeps.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $O/pytest_libgeeps.log)"; grep -E "FAILED" $O/pytest_libgeeps.log | head -20
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 200 python scripts/run_clock_bench.py 1 8388608 10 2 0 ipc $O/clock_p1_gather_$i.json > /dev/null 2>> $O/clock.err || exit 1
  GEEPS_DIRECT_READ=1 timeout -k 10 200 python scripts/run_clock_bench.py 1 8388608 10 2 0 ipc $O/clock_p1_direct_read_$i.json > /dev/null 2>> $O/clock.err || exit 1
done
for f in $O/clock_*.json; do echo "$(basename $f) $(cat $f)"; done
