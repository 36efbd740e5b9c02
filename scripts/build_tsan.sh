#!/bin/bash
# Host-only ThreadSanitizer build of libgeeps and the sum test app
# (build/tsan/), for `GEEPS_SUM_APP=build/tsan/geeps_sum_app pytest
# tests/test_libgeeps.py -m gpu`: libgeeps' own threads (per-client server
# readers, per-server client readers, server threads, the app thread) are
# instrumented; device code and the HIP runtime are not (libgp_reduce.so is the
# product build).  Both built by ROCm's clang (one TSan runtime).
# TSAN_OPTIONS=halt_on_error=1 makes the first report fatal.
set -e
REPO=$(cd "$(dirname "$0")/.." && pwd)
OUT=$REPO/build/tsan
mkdir -p "$OUT"
/opt/rocm/lib/llvm/bin/clang++ -O1 -g -std=c++17 -fPIC -Wall -Wno-sign-compare -pthread -fsanitize=thread -fno-omit-frame-pointer \
  -I"$REPO/include" -I"$REPO/geeps_amd/csrc/geeps" -shared -o "$OUT/libgeeps.so" \
  "$REPO"/geeps_amd/csrc/geeps/*.cpp -L"$REPO/geeps_amd/lib" -lgp_reduce \
  -Wl,-rpath,'$ORIGIN/../../geeps_amd/lib'
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -std=c++17 -I "$REPO/include" -Xarch_host -fsanitize=thread \
  "$REPO/tests/apps/geeps_sum_app.cpp" -o "$OUT/geeps_sum_app" -L"$OUT" -lgeeps \
  -Wl,-rpath,'$ORIGIN'
echo "built $OUT"
