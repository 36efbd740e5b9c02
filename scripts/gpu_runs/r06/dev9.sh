#!/bin/bash
# Round 6: libgeeps' pinned-buffer changes (TSan annotations, no-ops in this
# build; PinnedPool's acquire fence) and the row-plan declarations moved out of
# gp_kernels.hpp: the GPU suite and smoke, once.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r06/dev9
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -24 $OUT/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; exit $rc
