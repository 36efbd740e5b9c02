// r3_wave_tune.hip — round-3 probe 3 (tuning harness, not product code; it
// #includes the product kernels): the planned fused init and planned gather
// on a random index (70-74 % in the bench line against 76 % in
// the round-3 probes).  Both are row_wave_kernel over a destination-sorted
// residual: random 512-B source rows in, a front-to-back destination walk out.
// Variants of the wave-map kernel (wave_var_kernel): rows per 32-lane group in
// flight (8 = production, 16, 32: row pointers fetched by __shfl as needed
// instead of held in registers), cache policy of the random loads and of the
// sequential stores, blocks per CU.  Two allocation settings: fresh buffers,
// and buffers allocated after a 36-GiB allocation was freed (the bench's
// row-op leg runs after its headline arena).  Each variant is bit-checked
// against production before timing.  Usage: r3_wave_tune [rounds]
#include "../../geeps_amd/csrc/gp_reduce.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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

constexpr size_t R = 8u << 20, W = 128, N = R * W;

// OP kInitFrom (y[to] = 0 + x[from]) or kAssignTo (y[to] = x[from]); 128-float
// rows, whole rows, sorted destinations; RPG rows per group per burst.
template <int OP, int RPG, bool NTL, bool NTS>
__global__ __launch_bounds__(kBlock) void wave_var_kernel(float *__restrict__ y, const float *__restrict__ x,
                                                          const gp_double_index *__restrict__ index, size_t num_rows) {
  typedef __attribute__((address_space(1))) f4 GT;
  constexpr int LPR = 32, kG = 2, kRowsPerGroup = 32;
  const int wl = threadIdx.x & 63, lane = wl % LPR, gw = wl / LPR;
  const size_t wave = ((size_t)blockIdx.x * kBlock + threadIdx.x) / 64;
  const size_t wstride = (size_t)gridDim.x * (kBlock / 64) * 64;
  size_t t = wave * 64;
  if (t >= num_rows) return;
  uint64_t msrc = 0, mdst = 0;
  auto resolve = [&](const gp_double_index &ix, bool live) {
    msrc = mdst = 0;
    if (!live) return;
    uint64_t from, to;
    row_endpoints<OP>(ix, 0, 0, from, to);
    msrc = reinterpret_cast<uint64_t>(x + from * W);
    mdst = reinterpret_cast<uint64_t>(y + to * W);
  };
  {
    const bool live = t + wl < num_rows;
    gp_double_index ix = {0, 0};
    if (live) ix = index[t + wl];
    resolve(ix, live);
  }
  for (; t < num_rows; t += wstride) {
    const size_t nr = t + wstride + wl;
    const bool nlive = nr < num_rows;
    gp_double_index nix = {0, 0};
    if (nlive) nix = index[nr];
    const size_t rows_here = num_rows - t < 64 ? num_rows - t : 64;
    for (int i0 = 0; i0 < kRowsPerGroup; i0 += RPG) {
      f4 xs[RPG];
#pragma unroll
      for (int k = 0; k < RPG; ++k) {
        const int rt = gw + kG * (i0 + k);
        const uint64_t sp = shfl64(msrc, rt);
        if ((size_t)rt < rows_here) {
          const GT *p = reinterpret_cast<const GT *>(sp) + lane;
          xs[k] = NTL ? __builtin_nontemporal_load(p) : *p;
        }
      }
#pragma unroll
      for (int k = 0; k < RPG; ++k) {
        const int rt = gw + kG * (i0 + k);
        const uint64_t dp = shfl64(mdst, rt);
        if ((size_t)rt < rows_here) {
          GT *d = reinterpret_cast<GT *>(dp) + lane;
          const f4 v = OP == kInitFrom ? f4(0.0f) + xs[k] : xs[k];
          if (NTS)
            __builtin_nontemporal_store(v, d);
          else
            *d = v;
        }
      }
    }
    resolve(nix, nlive);
  }
}

__global__ void mismatch_kernel(const uint32_t *a, const uint32_t *b, size_t n, unsigned long long *cnt) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  unsigned long long c = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) c += a[i] != b[i];
  if (c) atomicAdd(cnt, c);
}

template <int OP, int RPG, bool NTL, bool NTS>
int resident() {
  static std::atomic<int> occ{0};
  return resident_blocks(reinterpret_cast<const void *>(&wave_var_kernel<OP, RPG, NTL, NTS>), occ);
}

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 5;
  std::mt19937_64 g(3);
  std::vector<uint64_t> perm(R);
  std::iota(perm.begin(), perm.end(), 0);
  std::shuffle(perm.begin(), perm.end(), g);
  std::vector<gp_double_index> srt(R), gat(R);
  for (size_t r = 0; r < R; ++r) {
    srt[perm[r]] = {r, perm[r]};  // init: y[id1] = 0 + x[id0], sorted by id1
    gat[r] = {r, perm[r]};        // gather: y[id0] = x[id1], sorted by id0
  }
  gp_double_index *isrt, *igat;
  CK(hipMalloc(&isrt, R * 16));
  CK(hipMalloc(&igat, R * 16));
  CK(hipMemcpy(isrt, srt.data(), R * 16, hipMemcpyHostToDevice));
  CK(hipMemcpy(igat, gat.data(), R * 16, hipMemcpyHostToDevice));
  unsigned long long *cnt;
  CK(hipMalloc(&cnt, 8));
  const size_t G = (size_t)num_cus();
  hipEvent_t ea, eb;
  CK(hipEventCreate(&ea));
  CK(hipEventCreate(&eb));

  for (int setting = 0; setting < 2; ++setting) {
    void *big = nullptr;
    if (setting == 1) {  // the bench's order: a 36-GiB arena first, freed before the row-op buffers
      CK(hipMalloc(&big, 36ull << 30));
      CK(hipMemset(big, 0, 36ull << 30));
      CK(hipDeviceSynchronize());
      CK(hipFree(big));
    }
    float *x, *y, *yr;
    CK(hipMalloc(&x, N * 4));
    CK(hipMalloc(&y, N * 4));
    CK(hipMalloc(&yr, N * 4));
    {
      std::vector<float> h(N);
      std::uniform_real_distribution<float> d(-0.5f, 0.5f);
      for (size_t i = 0; i < N; ++i) h[i] = d(g);
      CK(hipMemcpy(x, h.data(), N * 4, hipMemcpyHostToDevice));
      CK(hipMemset(y, 0, N * 4));
    }
    struct V {
      std::string name;
      std::function<void()> f;
      int op;
    };
    auto var = [&](auto kern, int occ, int per_cu) {
      return [=] {
        const size_t cap = G * (per_cu > 0 ? per_cu : occ);
        const size_t grid = std::min((R + kBlock - 1) / kBlock, cap);
        return std::make_pair(kern, grid);
      };
    };
    (void)var;
    std::vector<V> vs;
#define VAR(OPV, RPGV, NTLV, NTSV, PCU, NAME)                                                             \
  vs.push_back({NAME, [&] {                                                                               \
                  const int occ = resident<OPV, RPGV, NTLV, NTSV>();                                      \
                  const size_t cap = G * (PCU > 0 ? PCU : occ);                                           \
                  const size_t grid = std::min((R + kBlock - 1) / kBlock, cap);                           \
                  hipLaunchKernelGGL((wave_var_kernel<OPV, RPGV, NTLV, NTSV>), dim3((unsigned)grid),      \
                                     dim3(kBlock), 0, 0, y, x, OPV == kInitFrom ? isrt : igat, R);         \
                },                                                                                        \
                OPV});
    vs.push_back({"init prod (wave, sorted)", [&] { launch_row_op<kInitFrom>(y, x, isrt, R, {0, 0}, W, ~size_t(0), 0, true); }, kInitFrom});
    VAR(kInitFrom, 8, true, true, 0, "init var 8  ntl nts res")
    VAR(kInitFrom, 16, true, true, 0, "init var 16 ntl nts res")
    VAR(kInitFrom, 32, true, true, 0, "init var 32 ntl nts res")
    VAR(kInitFrom, 8, false, true, 0, "init var 8  pl  nts res")
    VAR(kInitFrom, 8, true, false, 0, "init var 8  ntl pst res")
    VAR(kInitFrom, 16, true, false, 0, "init var 16 ntl pst res")
    VAR(kInitFrom, 8, true, true, 2, "init var 8  ntl nts 2/CU")
    VAR(kInitFrom, 16, true, true, 2, "init var 16 ntl nts 2/CU")
    VAR(kInitFrom, 32, true, true, 2, "init var 32 ntl nts 2/CU")
    vs.push_back({"gath prod (wave, sorted)", [&] { launch_row_op<kAssignTo>(y, x, igat, R, {0, 0}, W, ~size_t(0), 0, true); }, kAssignTo});
    VAR(kAssignTo, 8, true, true, 0, "gath var 8  ntl nts res")
    VAR(kAssignTo, 16, true, true, 0, "gath var 16 ntl nts res")
    VAR(kAssignTo, 32, true, true, 0, "gath var 32 ntl nts res")
    VAR(kAssignTo, 8, false, true, 0, "gath var 8  pl  nts res")
    VAR(kAssignTo, 8, true, false, 0, "gath var 8  ntl pst res")
    VAR(kAssignTo, 16, true, true, 2, "gath var 16 ntl nts 2/CU")
    VAR(kAssignTo, 32, true, true, 2, "gath var 32 ntl nts 2/CU")
#undef VAR
    // checks against production
    for (auto &v : vs) {
      if (v.op == kInitFrom)
        launch_row_op<kInitFrom>(y, x, isrt, R, {0, 0}, W, ~size_t(0), 0, true);
      else
        launch_row_op<kAssignTo>(y, x, igat, R, {0, 0}, W, ~size_t(0), 0, true);
      CK(hipMemcpy(yr, y, N * 4, hipMemcpyDeviceToDevice));
      CK(hipMemset(y, 0x7f, N * 4));
      v.f();
      CK(hipMemset(cnt, 0, 8));
      hipLaunchKernelGGL(mismatch_kernel, dim3(1024), dim3(256), 0, 0, (const uint32_t *)y, (const uint32_t *)yr, N, cnt);
      unsigned long long h = 0;
      CK(hipMemcpy(&h, cnt, 8, hipMemcpyDeviceToHost));
      if (h) {
        std::printf("check %s: %llu mismatches\n", v.name.c_str(), h);
        return 3;
      }
    }
    std::vector<std::vector<float>> ms(vs.size());
    for (auto &v : vs) v.f();
    CK(hipDeviceSynchronize());
    for (int r = 0; r < rounds; ++r)
      for (size_t i = 0; i < vs.size(); ++i) {
        CK(hipEventRecord(ea, 0));
        vs[i].f();
        CK(hipEventRecord(eb, 0));
        CK(hipEventSynchronize(eb));
        float t = 0;
        CK(hipEventElapsedTime(&t, ea, eb));
        ms[i].push_back(t);
      }
    CK(hipGetLastError());
    std::printf("setting %d (%s)\n", setting, setting ? "after a freed 36-GiB allocation" : "fresh buffers");
    std::printf("%-28s %9s %9s %8s\n", "variant", "med_ms", "min_ms", "%8TB/s");
    const double bytes = 2.0 * N * 4 + 16.0 * R;
    for (size_t i = 0; i < vs.size(); ++i) {
      auto m = ms[i];
      std::sort(m.begin(), m.end());
      const double med = m[m.size() / 2];
      std::printf("%-28s %9.4f %9.4f %7.1f%%\n", vs[i].name.c_str(), med, m[0], 100.0 * bytes / (med * 1e-3) / 8e12);
    }
    CK(hipFree(x));
    CK(hipFree(y));
    CK(hipFree(yr));
  }
  return 0;
}
