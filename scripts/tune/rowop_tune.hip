// rowop_tune.hip — sweep of the product row-op kernel's template parameters
// (rows per group iteration, grid size) for the client
// scatter-add / gather at 8M RowData rows with a random-permutation index.
// Tuning harness, not product code: it #includes the product kernels.
#include "../../geeps_amd/csrc/gp_reduce.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <numeric>
#include <random>
#include <vector>

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e = (x);                                                                 \
    if (e != hipSuccess) {                                                              \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      std::exit(2);                                                                     \
    }                                                                                   \
  } while (0)

template <int OP, int LPR, int RPG>
void launch(float *y, const float *x, const gp_double_index *idx, size_t n, size_t W, int per_cu) {
  constexpr int kGroups = kBlock / LPR;
  const size_t groups = (n + RPG - 1) / RPG;
  size_t grid = (groups + kGroups - 1) / kGroups;
  const size_t cap = (size_t)num_cus() * per_cu;
  if (grid > cap) grid = cap;
  hipLaunchKernelGGL((row_op_kernel<f4, 4, OP, LPR, RPG>), dim3((unsigned)grid), dim3(kBlock), 0, 0,
                     y, x, idx, n, 0, 0, W, W / 4, (size_t)-1);
}

int main(int argc, char **argv) {
  const size_t R = argc > 1 ? std::strtoull(argv[1], 0, 10) : (1ull << 23);
  const size_t W = 128;
  const int rounds = argc > 2 ? std::atoi(argv[2]) : 5;
  float *x, *y;
  gp_double_index *idx;
  CK(hipMalloc(&x, R * W * 4));
  CK(hipMalloc(&y, R * W * 4));
  CK(hipMalloc(&idx, R * sizeof(gp_double_index)));
  CK(hipMemset(x, 0, R * W * 4));
  CK(hipMemset(y, 0, R * W * 4));
  std::vector<gp_double_index> h(R);
  std::vector<uint64_t> perm(R);
  std::iota(perm.begin(), perm.end(), 0);
  std::mt19937_64 rng(5);
  std::shuffle(perm.begin(), perm.end(), rng);
  for (size_t r = 0; r < R; ++r) h[r] = gp_double_index{r, perm[r]};
  CK(hipMemcpy(idx, h.data(), R * sizeof(gp_double_index), hipMemcpyHostToDevice));
  std::vector<gp_double_index> hid(R);
  for (size_t r = 0; r < R; ++r) hid[r] = gp_double_index{r, r};
  gp_double_index *ident;
  CK(hipMalloc(&ident, R * sizeof(gp_double_index)));
  CK(hipMemcpy(ident, hid.data(), R * sizeof(gp_double_index), hipMemcpyHostToDevice));

  struct V {
    const char *name;
    double bytes;
    std::function<void()> run;
    std::vector<float> ms;
  };
  const double add_b = 3.0 * R * W * 4 + 16.0 * R, gat_b = 2.0 * R * W * 4 + 16.0 * R;
  std::vector<V> vs;
#define ADD(NAME, B, ...) vs.push_back(V{NAME, B, [&]() { __VA_ARGS__; }, {}})
  // rows in flight per group (RPG) x blocks per CU, on the production kernel
  // (with its per-stream cache policy); production: add RPG 4, others RPG 8, 8/CU
  ADD("add   R2 x8", add_b, (launch<kAddFrom, 32, 2>(y, x, idx, R, W, 8)));
  ADD("add   R4 x4", add_b, (launch<kAddFrom, 32, 4>(y, x, idx, R, W, 4)));
  ADD("add   R4 x8 (prod)", add_b, (launch<kAddFrom, 32, 4>(y, x, idx, R, W, 8)));
  ADD("add   R4 x16", add_b, (launch<kAddFrom, 32, 4>(y, x, idx, R, W, 16)));
  ADD("add   R8 x4", add_b, (launch<kAddFrom, 32, 8>(y, x, idx, R, W, 4)));
  ADD("add   R8 x8", add_b, (launch<kAddFrom, 32, 8>(y, x, idx, R, W, 8)));
  ADD("gath  R4 x8", gat_b, (launch<kAssignTo, 32, 4>(y, x, idx, R, W, 8)));
  ADD("gath  R8 x4", gat_b, (launch<kAssignTo, 32, 8>(y, x, idx, R, W, 4)));
  ADD("gath  R8 x8 (prod)", gat_b, (launch<kAssignTo, 32, 8>(y, x, idx, R, W, 8)));
  ADD("gath  R8 x16", gat_b, (launch<kAssignTo, 32, 8>(y, x, idx, R, W, 16)));
  ADD("gath  R16 x4", gat_b, (launch<kAssignTo, 32, 16>(y, x, idx, R, W, 4)));
  ADD("gath  R16 x8", gat_b, (launch<kAssignTo, 32, 16>(y, x, idx, R, W, 8)));
  ADD("init  R4 x8", gat_b, (launch<kInitFrom, 32, 4>(y, x, idx, R, W, 8)));
  ADD("init  R8 x8 (prod)", gat_b, (launch<kInitFrom, 32, 8>(y, x, idx, R, W, 8)));
  ADD("init  R8 x16", gat_b, (launch<kInitFrom, 32, 8>(y, x, idx, R, W, 16)));
  ADD("init  R16 x8", gat_b, (launch<kInitFrom, 32, 16>(y, x, idx, R, W, 8)));
  ADD("add ident R4 x8 (prod)", add_b, (launch<kAddFrom, 32, 4>(y, x, ident, R, W, 8)));
  ADD("add ident R8 x8", add_b, (launch<kAddFrom, 32, 8>(y, x, ident, R, W, 8)));
  ADD("gath ident R8 x8 (prod)", gat_b, (launch<kAssignTo, 32, 8>(y, x, ident, R, W, 8)));
  ADD("gath ident R16 x8", gat_b, (launch<kAssignTo, 32, 16>(y, x, ident, R, W, 8)));

  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (auto &v : vs) v.run();
  CK(hipDeviceSynchronize());
  for (int r = 0; r < rounds; ++r)
    for (auto &v : vs) {
      CK(hipEventRecord(a));
      v.run();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      v.ms.push_back(ms);
    }
  std::printf("%-26s %10s %10s %10s %8s\n", "variant", "med_ms", "min_ms", "GB/s", "frac8T");
  for (auto &v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const double med = v.ms[v.ms.size() / 2];
    const double gbs = v.bytes / (med * 1e-3) / 1e9;
    std::printf("%-26s %10.4f %10.4f %10.1f %8.4f\n", v.name, med, v.ms[0], gbs, gbs / 8000.0);
  }
  return 0;
}
