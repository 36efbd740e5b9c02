#!/bin/bash
# Round 5, once: the randomized libgeeps campaign (300 seeds; round 5 draws
# host tiers and IPC faults too) and the parity fuzz campaign (the unplanned
# calls' check / map build / retirement changed), at the round's code.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r05campaign}; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u -m pytest tests/test_libgeeps.py -m gpu -v -k "ipc_failure or host_tier" --timeout 100 --timeout-method thread > $O/pytest_ipc_host.log 2>&1; rc=$?
echo "ipc/host rc=$rc $(tail -n 1 $O/pytest_ipc_host.log)"; grep -E "FAILED" $O/pytest_ipc_host.log | head; [ $rc -eq 0 ] || exit $rc
# the two seeds whose real IPC mis-mappings (and a failed export's lingering
# runtime error) failed the first campaign, first
GEEPS_STRESS_CASES=300 timeout -k 10 200 python -u -m pytest "tests/test_libgeeps.py::test_randomized_configurations[256]" "tests/test_libgeeps.py::test_randomized_configurations[285]" -m gpu -v -s --timeout 100 --timeout-method thread > $O/pytest_seeds.log 2>&1; rc=$?
echo "seeds rc=$rc $(tail -n 1 $O/pytest_seeds.log)"; [ $rc -eq 0 ] || exit $rc
GEEPS_STRESS_CASES=300 timeout -k 10 560 python -u -m pytest tests/test_libgeeps.py -m gpu -v -s -k "randomized" --timeout 250 --timeout-method thread > $O/pytest_stress.log 2>&1; rc=$?
echo "stress rc=$rc $(tail -n 1 $O/pytest_stress.log)"; grep -E "FAILED" $O/pytest_stress.log | head -20; [ $rc -eq 0 ] || exit $rc
GEEPS_FUZZ_CASES=2000 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "fuzz" --timeout 175 --timeout-method thread > $O/pytest_fuzz.log 2>&1; rc=$?
echo "fuzz rc=$rc $(tail -n 1 $O/pytest_fuzz.log)"; grep -E "FAILED" $O/pytest_fuzz.log | head; exit $rc
