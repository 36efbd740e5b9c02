#!/bin/bash
# Bucket-sum cache-policy probe (buffer-op aux bits) + bench with the same-box copy probe.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r25
timeout -k 10 300 ./build/tune/bucket_policy_tune 7 > gpurun_out/r25/policy.txt 2> gpurun_out/r25/policy.err; rc=$?
echo "policy rc=$rc"; cat gpurun_out/r25/policy.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-inclusive --no-rowops > gpurun_out/r25/bench.json 2> gpurun_out/r25/bench.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/r25/bench.json; exit $rc
