#!/bin/bash
# Tuning sweep of bucket-sum variants + PMC traffic passes on the bench kernel.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 ./scripts/tune/bucket_tune $((1<<20)) 1024 8 5 > gpurun_out/tune2.txt 2> gpurun_out/tune2.err; rc=$?
echo "tune rc=$rc"; cat gpurun_out/tune2.txt
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_$c" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-host-inclusive > "$GRAFT_REPO_ROOT/gpurun_out/pmc_$c.log" 2>&1; rc=$?
  echo "pmc $c rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
exit 0
