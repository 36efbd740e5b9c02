// Concurrency check of the C-ABI's host row ops (geeps_amd/csrc/gp_host.cpp)
// and their persistent worker pool, built with ThreadSanitizer by
// tests/test_host_rows.py (CPU only: gp_host.cpp has no device code).
//
// 6 threads, as libgeeps' app thread and reader threads would, each run 5
// rounds of large scatter-adds, fused inits, gathers, adds and zeroes on
// buffers of their own, and check every element against a serial loop.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "gp_reduce.h"

namespace gp_internal {
// gp_reduce.hip's error recorder; this harness links gp_host.cpp alone
int set_error(int code, const char *msg) {
  std::fprintf(stderr, "gp error %d: %s\n", code, msg);
  return code;
}
}  // namespace gp_internal

namespace {
constexpr size_t W = 128;

bool check_thread(unsigned seed) {
  std::mt19937_64 rng(seed);
  const size_t n = 12000 + seed * 37, cache = n + 500;  // >= 4 MiB of rows: the pool runs
  std::vector<gp_double_index> idx(n);
  std::vector<size_t> perm(cache);
  for (size_t i = 0; i < cache; ++i) perm[i] = i;
  std::shuffle(perm.begin(), perm.end(), rng);
  for (size_t i = 0; i < n; ++i) idx[i] = gp_double_index{i, perm[i]};
  idx[n / 2].id1 = idx[0].id1;  // one repeated destination
  std::uniform_real_distribution<float> u(-1.0f, 1.0f);
  std::vector<float> x(n * W), y(cache * W), want(cache * W), g(n * W), gwant(n * W);
  for (auto &v : x) v = u(rng);
  for (int round = 0; round < 5; ++round) {
    for (size_t i = 0; i < y.size(); ++i) y[i] = want[i] = (float)(i % 97) * 0.25f;
    if (gp_host_scatter_add_rows(y.data(), x.data(), idx.data(), n, gp_double_index{0, 0}, W, n * W) != GP_OK)
      return false;
    for (size_t i = 0; i < n; ++i)
      for (size_t v = 0; v < W; ++v) want[idx[i].id1 * W + v] += x[idx[i].id0 * W + v];
    if (std::memcmp(y.data(), want.data(), y.size() * sizeof(float)) != 0) return false;
    // the fused init: zerofy of the listed rows, then the add
    if (gp_host_scatter_init_rows(y.data(), x.data(), idx.data(), n, gp_double_index{0, 0}, W, n * W) != GP_OK)
      return false;
    for (size_t i = 0; i < n; ++i) std::memset(&want[idx[i].id1 * W], 0, W * sizeof(float));
    for (size_t i = 0; i < n; ++i)
      for (size_t v = 0; v < W; ++v) want[idx[i].id1 * W + v] += x[idx[i].id0 * W + v];
    if (std::memcmp(y.data(), want.data(), y.size() * sizeof(float)) != 0) return false;
    if (gp_host_gather_rows(g.data(), y.data(), idx.data(), n, gp_double_index{0, 0}, W, n * W) != GP_OK)
      return false;
    for (size_t i = 0; i < n; ++i) std::memcpy(&gwant[idx[i].id0 * W], &y[idx[i].id1 * W], W * sizeof(float));
    if (std::memcmp(g.data(), gwant.data(), g.size() * sizeof(float)) != 0) return false;
    if (gp_host_add(y.size(), y.data(), want.data()) != GP_OK) return false;
    for (size_t i = 0; i < y.size(); ++i)
      if (y[i] != want[i] + want[i]) return false;
    if (gp_host_zero(y.size(), y.data()) != GP_OK) return false;
    for (float v : y)
      if (v != 0.0f) return false;
  }
  return true;
}
}  // namespace

int main() {
  std::vector<std::thread> ts;
  std::vector<int> ok(6, 0);
  for (unsigned t = 0; t < ok.size(); ++t) ts.emplace_back([t, &ok] { ok[t] = check_thread(t + 1); });
  for (auto &t : ts) t.join();
  for (int v : ok)
    if (!v) {
      std::printf("mismatch\n");
      return 1;
    }
  std::printf("ok\n");
  return 0;
}
