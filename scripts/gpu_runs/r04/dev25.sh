#!/bin/bash
# Round 4: per-client server copy streams and staged refreshes landed outside
# the channel lock: the libgeeps tests, then the one-GPU rehearsal of the
# multi-GPU bench leg (2 processes, both tables, staged and in place).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04dev25}; mkdir -p $O
GEEPS_STRESS_CASES=40 timeout -k 10 600 python -u -m pytest tests/test_libgeeps.py -m gpu -v --timeout 175 --timeout-method thread > $O/pytest_libgeeps.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $O/pytest_libgeeps.log)"; grep -E "FAILED" $O/pytest_libgeeps.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -c "import json, bench; print(json.dumps(bench.libgeeps_multi_gpu_leg(2, 1 << 20, 1024, gpus_seen=1)))" > $O/multi_rehearsal.json 2> $O/multi_rehearsal.err; rc=$?
echo "rehearsal rc=$rc"; cat $O/multi_rehearsal.json; exit $rc
