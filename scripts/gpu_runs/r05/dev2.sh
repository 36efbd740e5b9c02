#!/bin/bash
# r05 dev2: one peer copy per staged / socket refresh (shard buffers swapped
# with the reader's landing buffer): the libgeeps tests, the configs[2] rank
# tests, then the one-GPU rehearsal of the multi-GPU bench leg.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r05dev2}; mkdir -p $O
export PYTHONUNBUFFERED=1
GEEPS_STRESS_CASES=40 timeout -k 10 700 python -u -m pytest tests/test_libgeeps.py tests/test_rccl.py -m gpu -v --timeout 175 --timeout-method thread > $O/pytest_libgeeps.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $O/pytest_libgeeps.log)"; grep -E "FAILED" $O/pytest_libgeeps.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -c "import json, bench; print(json.dumps(bench.libgeeps_multi_gpu_leg(2, 1 << 20, 1024, gpus_seen=1)))" > $O/multi_rehearsal.json 2> $O/multi_rehearsal.err; rc=$?
echo "rehearsal rc=$rc"; cat $O/multi_rehearsal.json; exit $rc
