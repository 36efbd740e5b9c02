#!/bin/bash
# Round 4: HBM traffic of the unplanned steady state (inverse-map walk, ranges
# gather, device check): two rocprofv3 --pmc passes, one counter each.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04dev26}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o run -- python3 $GRAFT_REPO_ROOT/scripts/probes/steady_rowops.py > $O/fetch.out 2> $O/fetch.err; rc=$?
echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o run -- python3 $GRAFT_REPO_ROOT/scripts/probes/steady_rowops.py > $O/write.out 2> $O/write.err; rc=$?
echo "write rc=$rc"; exit $rc
