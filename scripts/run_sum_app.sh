#!/bin/bash
# Debug driver: run tests/apps/geeps_sum_app as P local processes with each
# process's stdout/stderr in OUTDIR/p<id>.{out,err}; every process under its own
# time limit.  Usage: run_sum_app.sh OUTDIR SECONDS TRANSPORT P rows clocks slack channels rmw mode [spec]
out=$1; lim=$2; tr=$3; P=$4; shift 4
mkdir -p "$out"
base=$(( 20000 + (RANDOM % 700) * 16 ))  # below the ephemeral port range (32768+)
pids=()
for ((p = 0; p < P; p++)); do
  GEEPS_TRANSPORT=$tr timeout -k 5 "$lim" "$GRAFT_REPO_ROOT/build/tests/geeps_sum_app" "$p" "$P" "$base" "$@" \
    > "$out/p$p.out" 2> "$out/p$p.err" &
  pids+=($!)
done
rc=0
for ((p = 0; p < P; p++)); do
  wait "${pids[$p]}"; r=$?
  echo "p$p rc=$r $(head -c 200 "$out/p$p.out")"
  [ $r -eq 0 ] || rc=$r
done
exit $rc
