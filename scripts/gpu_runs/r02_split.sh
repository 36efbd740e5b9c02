#!/bin/bash
# Round 2: big/small sweep split that avoids tile-major rests: GPU suite, then
# the per-rank scaling emulation (N = 1/2/4/8, two passes).
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r02p2; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $O/pytest_gpu.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/pytest_gpu.log | head -20; exit $rc; }
ARGS="--no-cpu-baseline --no-host-inclusive --no-rowops --no-e2e --no-config2 --no-hbm-probe --steps 20 --warmup 3"
for rep in 1 2; do
  for n in 1 2 4 8; do
    timeout -k 10 120 python bench.py $ARGS --rows $((1048576 / n)) > $O/emul_n${n}_r$rep.json 2> $O/emul_n${n}_r$rep.err; rc=$?
    echo "n=$n rep=$rep rc=$rc $(python3 -c "import json;d=json.load(open('$O/emul_n${n}_r$rep.json'));r=d['roofline'];print(d['ms_per_step'], r['frac'], r['launches_per_step'], r['other_launches_per_step'])")"; [ $rc -eq 0 ] || exit $rc
  done
done
