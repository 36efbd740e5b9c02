#!/bin/bash
# Host-only UndefinedBehaviorSanitizer build of libgeeps and the sum test app
# (build/ubsan/), for `GEEPS_SUM_APP=build/ubsan/geeps_sum_app pytest
# tests/test_libgeeps.py -m gpu`.  Device code is untouched: libgp_reduce.so
# is the product build (geeps_amd/lib); UBSan aborts on the first report.
set -e
REPO=$(cd "$(dirname "$0")/.." && pwd)
OUT=$REPO/build/ubsan
mkdir -p "$OUT"
g++ -O1 -g -std=c++17 -fPIC -Wall -Wno-sign-compare -pthread -fsanitize=undefined \
  -fno-sanitize-recover=undefined -fno-omit-frame-pointer \
  -I"$REPO/include" -I"$REPO/geeps_amd/csrc/geeps" -shared -o "$OUT/libgeeps.so" \
  "$REPO"/geeps_amd/csrc/geeps/*.cpp -L"$REPO/geeps_amd/lib" -lgp_reduce \
  -Wl,-rpath,'$ORIGIN/../../geeps_amd/lib'
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -std=c++17 -I "$REPO/include" \
  "$REPO/tests/apps/geeps_sum_app.cpp" -o "$OUT/geeps_sum_app" -L"$OUT" -lgeeps \
  -Wl,-rpath,'$ORIGIN'
echo "built $OUT"
