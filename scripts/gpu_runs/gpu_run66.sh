#!/bin/bash
# Config 2 line (2 clients) and the host-inclusive leg on the current build.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r66; mkdir -p $O
timeout -k 10 300 python bench.py --clients 2 --no-rowops > $O/bench_2clients.json 2> $O/bench_2clients.err; rc=$?
echo "bench 2 clients rc=$rc $(grep -o '"frac": [0-9.]*' $O/bench_2clients.json | head -1) $(grep -o '"avg_kernel_ms": [0-9.]*' $O/bench_2clients.json | head -1) $(grep -o '"delta_GBps": [0-9.]*' $O/bench_2clients.json)"; exit $rc
