// rownt_tune.hip — cache policy of the row-op kernel's streams (tuning harness,
// not product code; it #includes the product kernels).  The bucket sum gained
// 4-5 % from non-temporal bucket loads; the row ops use plain loads and stores.
// Here the production lane/row mapping (LPR lanes per row, RPG rows in flight)
// with nt on the x loads (L), the y loads of the scatter-add (Y) and the y
// stores (S), for gather / scatter-add / fused init at 128-float rows, 8 M rows
// (4 GiB), random-permutation and identity DoubleIndex.  "prod" is the product
// kernel (nt x loads in scatter-add and init since this probe), "plain" no nt.
// Usage: rownt_tune [rounds]
#include "../../geeps_amd/csrc/gp_reduce.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <numeric>
#include <random>
#include <string>
#include <vector>

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e = (x);                                                                 \
    if (e != hipSuccess) {                                                              \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      std::exit(2);                                                                     \
    }                                                                                   \
  } while (0)

template <int OP, int LPR, int RPG, int POL>
__global__ __launch_bounds__(kBlock) void row_nt(float *__restrict__ y, const float *__restrict__ x,
                                                 const gp_double_index *__restrict__ index,
                                                 size_t num_rows, size_t vw) {
  constexpr int kGroups = kBlock / LPR;
  const int lane = threadIdx.x % LPR;
  const size_t group = (size_t)blockIdx.x * kGroups + threadIdx.x / LPR;
  const size_t gstride = (size_t)gridDim.x * kGroups * RPG;
  f4 *yv = reinterpret_cast<f4 *>(y);
  const f4 *xv = reinterpret_cast<const f4 *>(x);
  for (size_t r0 = group * RPG; r0 < num_rows; r0 += gstride) {
    uint64_t from[RPG], to[RPG];
    bool live[RPG];
#pragma unroll
    for (int k = 0; k < RPG; ++k) {
      const size_t r = r0 + k;
      live[k] = r < num_rows;
      from[k] = to[k] = 0;
      if (live[k]) row_endpoints<OP>(index[r], 0, 0, from[k], to[k]);
    }
    for (size_t j = lane; j < vw; j += LPR) {
      f4 xs[RPG], ys[RPG];
#pragma unroll
      for (int k = 0; k < RPG; ++k)
        if (live[k]) xs[k] = (POL & 1) ? __builtin_nontemporal_load(xv + from[k] * vw + j) : xv[from[k] * vw + j];
      if (OP == kAddFrom) {
#pragma unroll
        for (int k = 0; k < RPG; ++k)
          if (live[k]) ys[k] = (POL & 2) ? __builtin_nontemporal_load(yv + to[k] * vw + j) : yv[to[k] * vw + j];
      }
#pragma unroll
      for (int k = 0; k < RPG; ++k) {
        if (!live[k]) continue;
        const f4 v = OP == kAddFrom ? ys[k] + xs[k] : (OP == kInitFrom ? f4(0.0f) + xs[k] : xs[k]);
        if (POL & 4) __builtin_nontemporal_store(v, yv + to[k] * vw + j);
        else yv[to[k] * vw + j] = v;
      }
    }
  }
}

template <int OP, int POL>
void launch_nt(float *y, const float *x, const gp_double_index *idx, size_t n) {
  constexpr int LPR = 32, RPG = OP == kAddFrom ? 4 : 8;
  constexpr int kGroups = kBlock / LPR;
  size_t grid = ((n + RPG - 1) / RPG + kGroups - 1) / kGroups;
  if (grid > grid_cap()) grid = grid_cap();
  hipLaunchKernelGGL((row_nt<OP, LPR, RPG, POL>), dim3((unsigned)grid), dim3(kBlock), 0, 0, y, x, idx, n,
                     (size_t)32);
}

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 7;
  const size_t bytes = 4ull << 30, R = bytes / 512;
  float *x, *y, *y2;
  CK(hipMalloc(&x, bytes));
  CK(hipMalloc(&y, bytes));
  CK(hipMalloc(&y2, bytes));
  std::vector<float> hx(1 << 24);
  for (size_t i = 0; i < hx.size(); ++i) hx[i] = (float)(i % 977) * 0.25f - 100.0f;
  for (size_t off = 0; off < bytes / 4; off += hx.size())
    CK(hipMemcpy(x + off, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
  std::vector<uint64_t> perm(R);
  std::iota(perm.begin(), perm.end(), 0);
  std::mt19937_64 rng(5);
  std::shuffle(perm.begin(), perm.end(), rng);
  std::vector<gp_double_index> h(R);
  gp_double_index *rnd, *ident;
  CK(hipMalloc(&rnd, R * 16));
  CK(hipMalloc(&ident, R * 16));
  for (size_t r = 0; r < R; ++r) h[r] = gp_double_index{r, perm[r]};
  CK(hipMemcpy(rnd, h.data(), R * 16, hipMemcpyHostToDevice));
  for (size_t r = 0; r < R; ++r) h[r] = gp_double_index{r, r};
  CK(hipMemcpy(ident, h.data(), R * 16, hipMemcpyHostToDevice));

  {  // correctness: all-nt forms == product
    CK(hipMemset(y, 0, bytes));
    CK(hipMemset(y2, 0, bytes));
    gp_gather_rows(y, x, rnd, R, {0, 0}, 128, (size_t)-1, nullptr);
    launch_nt<kAssignTo, 7>(y2, x, rnd, R);
    gp_scatter_add_rows(y, x, rnd, R, {0, 0}, 128, (size_t)-1, nullptr);
    launch_nt<kAddFrom, 7>(y2, x, rnd, R);
    CK(hipDeviceSynchronize());
    std::vector<float> a(1 << 24), b(1 << 24);
    size_t bad = 0;
    for (size_t off = 0; off < bytes / 4; off += a.size()) {
      CK(hipMemcpy(a.data(), y + off, a.size() * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(b.data(), y2 + off, b.size() * 4, hipMemcpyDeviceToHost));
      bad += std::memcmp(a.data(), b.data(), a.size() * 4) != 0;
    }
    std::printf("nt forms vs product: %zu mismatching 64-MiB blocks\n", bad);
  }

  struct V {
    std::string name;
    double bytes;
    std::function<void()> run;
    std::vector<float> ms;
  };
  std::vector<V> vs;
  const double gat_b = 2.0 * bytes + 16.0 * R, add_b = 3.0 * bytes + 16.0 * R;
  for (int which = 0; which < 2; ++which) {
    const gp_double_index *ix = which ? ident : rnd;
    const std::string tag = which ? "ident " : "random ";
    vs.push_back(V{tag + "gather prod", gat_b, [=]() { gp_gather_rows(y, x, ix, R, {0, 0}, 128, (size_t)-1, nullptr); }, {}});
    vs.push_back(V{tag + "gather plain", gat_b, [=]() { launch_nt<kAssignTo, 0>(y, x, ix, R); }, {}});
    vs.push_back(V{tag + "gather L", gat_b, [=]() { launch_nt<kAssignTo, 1>(y, x, ix, R); }, {}});
    vs.push_back(V{tag + "gather S", gat_b, [=]() { launch_nt<kAssignTo, 4>(y, x, ix, R); }, {}});
    vs.push_back(V{tag + "gather LS", gat_b, [=]() { launch_nt<kAssignTo, 5>(y, x, ix, R); }, {}});
    vs.push_back(V{tag + "add prod", add_b, [=]() { gp_scatter_add_rows(y, x, ix, R, {0, 0}, 128, (size_t)-1, nullptr); }, {}});
    vs.push_back(V{tag + "add plain", add_b, [=]() { launch_nt<kAddFrom, 0>(y, x, ix, R); }, {}});
    vs.push_back(V{tag + "add L", add_b, [=]() { launch_nt<kAddFrom, 1>(y, x, ix, R); }, {}});
    vs.push_back(V{tag + "add LY", add_b, [=]() { launch_nt<kAddFrom, 3>(y, x, ix, R); }, {}});
    vs.push_back(V{tag + "add LS", add_b, [=]() { launch_nt<kAddFrom, 5>(y, x, ix, R); }, {}});
    vs.push_back(V{tag + "add LYS", add_b, [=]() { launch_nt<kAddFrom, 7>(y, x, ix, R); }, {}});
    vs.push_back(V{tag + "init prod", gat_b, [=]() { gp_scatter_init_rows(y, x, ix, R, {0, 0}, 128, (size_t)-1, nullptr); }, {}});
    vs.push_back(V{tag + "init plain", gat_b, [=]() { launch_nt<kInitFrom, 0>(y, x, ix, R); }, {}});
    vs.push_back(V{tag + "init L", gat_b, [=]() { launch_nt<kInitFrom, 1>(y, x, ix, R); }, {}});
    vs.push_back(V{tag + "init LS", gat_b, [=]() { launch_nt<kInitFrom, 5>(y, x, ix, R); }, {}});
  }
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
  std::printf("%-22s %10s %10s %10s %8s\n", "variant", "med_ms", "min_ms", "GB/s", "frac8T");
  for (auto &v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const double med = v.ms[v.ms.size() / 2];
    const double gbs = v.bytes / (med * 1e-3) / 1e9;
    std::printf("%-22s %10.4f %10.4f %10.1f %8.4f\n", v.name.c_str(), med, v.ms[0], gbs, gbs / 8000.0);
  }
  return 0;
}
