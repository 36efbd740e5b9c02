// r3_isweep_tune.hip — round-3 probe 5 (tuning harness, not product code; it
// #includes the product kernels): a wave-local indexed sweep for the planned
// fused init and gather on a random index (>= 75 % of 8 TB/s;
// production row_wave_kernel runs 73.5-76.7 % across boxes).
//
// Probe 4 (r3_rand_tune) found random 512-B row reads at 97 % of the
// sequential read rate: the loss is the read/write mix, which the sweep sums
// avoid by phases (read a chunk, then write it).  Probe 1's indexed sweep
// (row_sweep_kernel) staged each block's index entries in LDS behind a block
// barrier before any row load, and ran 4-5 % under the dense sweep even on an
// identity index.  This one keeps everything per wave: lane l loads plan entry
// l of each 64-entry set of its 128-row slice (two coalesced 1-KiB reads), row
// pointers move by __shfl, rows are read in bursts of TG row pairs (a 32-lane
// half per row, 16 B per lane), parked in the wave's own 40-KiB LDS region
// (80 rows) and in registers (48 rows), then written to their destinations in
// plan order.  No block barrier; one block (4 waves, 160 KiB LDS) per CU; a
// launch moves 128 rows per wave, 64 MiB over 256 CUs.  PF: before its write
// phase a wave loads its slot's index entries of the NEXT launch, so they sit
// in L2 / MALL when that launch starts.
// Every variant is bit-checked against the production planned call.
// Probe 7 (psweep_kernel): the same slices in one persistent launch, the next
// slice's index entries loaded under this slice's writes.
// Usage: r3_isweep_tune [rounds]
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
#define GK(x)                                                            \
  do {                                                                   \
    int r_ = (x);                                                        \
    if (r_ != GP_OK) {                                                   \
      std::fprintf(stderr, "%s:%d %s -> %d\n", __FILE__, __LINE__, #x, r_); \
      std::exit(2);                                                      \
    }                                                                    \
  } while (0)

constexpr size_t R = 8u << 20, W = 128, N = R * W;
constexpr uint64_t kNone = ~0ull;
constexpr int kWaveRows = 128;  // plan entries per wave per launch
constexpr int kLdsRows = 80;    // of them parked in LDS (40 KiB per wave, 160 KiB per block)
constexpr int kPairs = kWaveRows / 2, kLdsPairs = kLdsRows / 2, kRegPairs = kPairs - kLdsPairs;

// OP kInitFrom (y[to] = 0.0f + x[from]) or kAssignTo (y[to] = x[from], from =
// id1, to = id0); 128-float rows, no limit.
template <int OP, int TG, bool PF>
__global__ __launch_bounds__(kBlock) void isweep_kernel(float *__restrict__ y, const float *__restrict__ x,
                                                        const gp_double_index *__restrict__ index,
                                                        size_t n_rows, size_t chunk) {
  typedef __attribute__((address_space(1))) f4 GT;
  static_assert(kPairs % TG == 0, "whole bursts");
  __shared__ f4 lds[4][kLdsRows * 32];
  const int wv = threadIdx.x / 64, wl = threadIdx.x % 64, lane = wl % 32, gw = wl / 32;
  const size_t waves = (size_t)gridDim.x * 4;
  const size_t slot = (size_t)blockIdx.x * 4 + wv;
  const size_t base = (chunk * waves + slot) * kWaveRows;
  if (base >= n_rows) return;
  uint64_t src[2], dst[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const size_t e = base + k * 64 + wl;
    src[k] = dst[k] = kNone;
    if (e < n_rows) {
      const gp_double_index ix = index[e];
      uint64_t from, to;
      row_endpoints<OP>(ix, 0, 0, from, to);
      src[k] = reinterpret_cast<uint64_t>(x + from * W);
      dst[k] = reinterpret_cast<uint64_t>(y + to * W);
    }
  }
  f4 keep[kRegPairs];
#pragma unroll
  for (int p0 = 0; p0 < kPairs; p0 += TG) {
    f4 v[TG];
#pragma unroll
    for (int j = 0; j < TG; ++j) {
      const int p = p0 + j, r = 2 * p;  // row r + gw of the slice: lane (r % 64) + gw of set r / 64
      const uint64_t sp = shfl64(src[r / 64], (r % 64) + gw);
      v[j] = f4(0.0f);
      if (sp != kNone) v[j] = __builtin_nontemporal_load(reinterpret_cast<const GT *>(sp) + lane);
    }
#pragma unroll
    for (int j = 0; j < TG; ++j) {
      const int p = p0 + j;
      const f4 val = OP == kInitFrom ? f4(0.0f) + v[j] : v[j];
      if (p < kLdsPairs)
        lds[wv][(2 * p + gw) * 32 + lane] = val;
      else
        keep[p >= kLdsPairs ? p - kLdsPairs : 0] = val;
    }
  }
  gp_double_index nx0 = {0, 0}, nx1 = {0, 0};
  if (PF) {  // this slot's entries of the next launch, into L2 / MALL
    const size_t nb = base + waves * kWaveRows;
    if (nb + wl < n_rows) nx0 = index[nb + wl];
    if (nb + 64 + wl < n_rows) nx1 = index[nb + 64 + wl];
  }
#pragma unroll
  for (int p = 0; p < kPairs; ++p) {
    const int r = 2 * p;
    const uint64_t dp = shfl64(dst[r / 64], (r % 64) + gw);
    if (dp != kNone)
      __builtin_nontemporal_store(p < kLdsPairs ? lds[wv][(2 * p + gw) * 32 + lane]
                                                : keep[p >= kLdsPairs ? p - kLdsPairs : 0],
                                  reinterpret_cast<GT *>(dp) + lane);
  }
  if (PF) asm volatile("" ::"v"(nx0.id0), "v"(nx1.id0));
}

// Persistent form (probe 7): each wave loops over slices wave, wave + waves,
// ... of 128 plan entries; the next slice's entries load into registers while
// this slice's rows are written, so no slice waits for a dependent index load
// (the launch-start bubble of isweep_kernel).  One launch.
template <int OP, int TG>
__global__ __launch_bounds__(kBlock) void psweep_kernel(float *__restrict__ y, const float *__restrict__ x,
                                                        const gp_double_index *__restrict__ index,
                                                        size_t n_rows) {
  typedef __attribute__((address_space(1))) f4 GT;
  static_assert(kPairs % TG == 0, "whole bursts");
  __shared__ f4 lds[4][kLdsRows * 32];
  const int wv = threadIdx.x / 64, wl = threadIdx.x % 64, lane = wl % 32, gw = wl / 32;
  const size_t waves = (size_t)gridDim.x * 4;
  const size_t stride = waves * kWaveRows;
  size_t base = ((size_t)blockIdx.x * 4 + wv) * kWaveRows;
  if (base >= n_rows) return;
  auto resolve = [&](size_t b, uint64_t *src, uint64_t *dst) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const size_t e = b + k * 64 + wl;
      src[k] = dst[k] = kNone;
      if (e < n_rows) {
        const gp_double_index ix = index[e];
        uint64_t from, to;
        row_endpoints<OP>(ix, 0, 0, from, to);
        src[k] = reinterpret_cast<uint64_t>(x + from * W);
        dst[k] = reinterpret_cast<uint64_t>(y + to * W);
      }
    }
  };
  uint64_t src[2], dst[2];
  resolve(base, src, dst);
  for (; base < n_rows; base += stride) {
    f4 keep[kRegPairs];
#pragma unroll
    for (int p0 = 0; p0 < kPairs; p0 += TG) {
      f4 v[TG];
#pragma unroll
      for (int j = 0; j < TG; ++j) {
        const int p = p0 + j, r = 2 * p;
        const uint64_t sp = shfl64(src[r / 64], (r % 64) + gw);
        v[j] = f4(0.0f);
        if (sp != kNone) v[j] = __builtin_nontemporal_load(reinterpret_cast<const GT *>(sp) + lane);
      }
#pragma unroll
      for (int j = 0; j < TG; ++j) {
        const int p = p0 + j;
        const f4 val = OP == kInitFrom ? f4(0.0f) + v[j] : v[j];
        if (p < kLdsPairs)
          lds[wv][(2 * p + gw) * 32 + lane] = val;
        else
          keep[p >= kLdsPairs ? p - kLdsPairs : 0] = val;
      }
    }
    uint64_t nsrc[2], ndst[2];
    resolve(base + stride, nsrc, ndst);  // the next slice's entries, under this slice's writes
#pragma unroll
    for (int p = 0; p < kPairs; ++p) {
      const int r = 2 * p;
      const uint64_t dp = shfl64(dst[r / 64], (r % 64) + gw);
      if (dp != kNone)
        __builtin_nontemporal_store(p < kLdsPairs ? lds[wv][(2 * p + gw) * 32 + lane]
                                                  : keep[p >= kLdsPairs ? p - kLdsPairs : 0],
                                    reinterpret_cast<GT *>(dp) + lane);
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      src[k] = nsrc[k];
      dst[k] = ndst[k];
    }
  }
}

template <int OP, int TG>
void launch_psweep(float *y, const float *x, const gp_double_index *ix, size_t n) {
  const size_t G = (size_t)num_cus();
  hipLaunchKernelGGL((psweep_kernel<OP, TG>), dim3((unsigned)G), dim3(kBlock), 0, 0, y, x, ix, n);
}

__global__ void mismatch_kernel(const uint32_t *a, const uint32_t *b, size_t n, unsigned long long *cnt) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  unsigned long long c = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) c += a[i] != b[i];
  if (c) atomicAdd(cnt, c);
}

template <int OP, int TG, bool PF>
void launch_isweep(float *y, const float *x, const gp_double_index *ix, size_t n) {
  const size_t G = (size_t)num_cus();
  const size_t per = G * 4 * kWaveRows;
  for (size_t c = 0; c * per < n; ++c)
    hipLaunchKernelGGL((isweep_kernel<OP, TG, PF>), dim3((unsigned)G), dim3(kBlock), 0, 0, y, x, ix, n, c);
}

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 5;
  std::mt19937_64 g(5);
  std::vector<uint64_t> perm(R);
  std::iota(perm.begin(), perm.end(), 0);
  std::shuffle(perm.begin(), perm.end(), g);
  // plans: destination-sorted, as a plan's residual is
  //   gather y[id0] = x[id1]: {i, perm[i]}       init y[id1] = 0 + x[id0]: {perm[d], d}
  std::vector<gp_double_index> gat(R), ini(R), ident(R);
  for (size_t r = 0; r < R; ++r) {
    gat[r] = {r, perm[r]};
    ini[r] = {perm[r], r};
    ident[r] = {r, r};
  }
  gp_double_index *igat, *iini, *iident;
  CK(hipMalloc(&igat, R * 16));
  CK(hipMalloc(&iini, R * 16));
  CK(hipMalloc(&iident, R * 16));
  CK(hipMemcpy(igat, gat.data(), R * 16, hipMemcpyHostToDevice));
  CK(hipMemcpy(iini, ini.data(), R * 16, hipMemcpyHostToDevice));
  CK(hipMemcpy(iident, ident.data(), R * 16, hipMemcpyHostToDevice));
  gp_row_plan pg, pi, pid;
  GK(gp_gather_plan_create(&pg, gat.data(), R, {0, 0}, W, ~size_t(0)));
  GK(gp_row_plan_create(&pi, ini.data(), R, {0, 0}, W, ~size_t(0)));
  GK(gp_gather_plan_create(&pid, ident.data(), R, {0, 0}, W, ~size_t(0)));
  unsigned long long *cnt;
  CK(hipMalloc(&cnt, 8));
  float *x, *y, *yr;
  CK(hipMalloc(&x, N * 4));
  CK(hipMalloc(&y, N * 4));
  CK(hipMalloc(&yr, N * 4));
  {
    std::vector<float> h(N);
    std::uniform_real_distribution<float> d(-0.5f, 0.5f);
    for (size_t i = 0; i < N; ++i) h[i] = d(g);
    for (size_t i = 0; i < N; i += 97) h[i] = -0.0f;  // the init's 0.0f + x turns these into +0
    CK(hipMemcpy(x, h.data(), N * 4, hipMemcpyHostToDevice));
  }
  struct V {
    std::string name;
    std::function<void()> f;
    int check;  // 1 gather (vs prod gather), 2 init (vs prod init), 3 identity gather (vs copy)
  };
  std::vector<V> vs;
  vs.push_back({"gath prod (wave, plan)", [&] { gp_gather_rows_planned(y, x, pg, 0); }, 1});
  vs.push_back({"gath isweep TG8", [&] { launch_isweep<kAssignTo, 8, false>(y, x, igat, R); }, 1});
  vs.push_back({"gath isweep TG16", [&] { launch_isweep<kAssignTo, 16, false>(y, x, igat, R); }, 1});
  vs.push_back({"gath isweep TG32", [&] { launch_isweep<kAssignTo, 32, false>(y, x, igat, R); }, 1});
  vs.push_back({"gath isweep TG8  PF", [&] { launch_isweep<kAssignTo, 8, true>(y, x, igat, R); }, 1});
  vs.push_back({"gath isweep TG16 PF", [&] { launch_isweep<kAssignTo, 16, true>(y, x, igat, R); }, 1});
  vs.push_back({"gath isweep TG32 PF", [&] { launch_isweep<kAssignTo, 32, true>(y, x, igat, R); }, 1});
  vs.push_back({"gath psweep TG16", [&] { launch_psweep<kAssignTo, 16>(y, x, igat, R); }, 1});
  vs.push_back({"gath psweep TG32", [&] { launch_psweep<kAssignTo, 32>(y, x, igat, R); }, 1});
  vs.push_back({"init prod (wave, plan)", [&] { gp_scatter_init_rows_planned(y, x, pi, 0); }, 2});
  vs.push_back({"init psweep TG32", [&] { launch_psweep<kInitFrom, 32>(y, x, iini, R); }, 2});
  vs.push_back({"init isweep TG16", [&] { launch_isweep<kInitFrom, 16, false>(y, x, iini, R); }, 2});
  vs.push_back({"init isweep TG16 PF", [&] { launch_isweep<kInitFrom, 16, true>(y, x, iini, R); }, 2});
  vs.push_back({"init isweep TG32 PF", [&] { launch_isweep<kInitFrom, 32, true>(y, x, iini, R); }, 2});
  vs.push_back({"ident copy prod (dense sweep)", [&] { gp_gather_rows_planned(y, x, pid, 0); }, 3});
  vs.push_back({"ident isweep TG16", [&] { launch_isweep<kAssignTo, 16, false>(y, x, iident, R); }, 3});
  vs.push_back({"ident isweep TG16 PF", [&] { launch_isweep<kAssignTo, 16, true>(y, x, iident, R); }, 3});
  vs.push_back({"ident psweep TG32", [&] { launch_psweep<kAssignTo, 32>(y, x, iident, R); }, 3});

  for (int c = 1; c <= 3; ++c) {
    if (c == 1) GK(gp_gather_rows_planned(yr, x, pg, 0));
    if (c == 2) GK(gp_scatter_init_rows_planned(yr, x, pi, 0));
    if (c == 3) GK(gp_gather_rows_planned(yr, x, pid, 0));
    CK(hipDeviceSynchronize());
    for (auto &v : vs) {
      if (v.check != c) continue;
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
  }
  std::printf("checks ok\n");
  hipEvent_t ea, eb;
  CK(hipEventCreate(&ea));
  CK(hipEventCreate(&eb));
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
  std::printf("8M rows x 512 B; bytes = 2 x rows + 16 B index per row\n");
  std::printf("%-30s %9s %9s %8s\n", "variant", "med_ms", "min_ms", "%8TB/s");
  const double bytes = 2.0 * N * 4 + 16.0 * R;
  for (size_t i = 0; i < vs.size(); ++i) {
    auto m = ms[i];
    std::sort(m.begin(), m.end());
    const double med = m[m.size() / 2];
    std::printf("%-30s %9.4f %9.4f %7.1f%%\n", vs[i].name.c_str(), med, m[0], 100.0 * bytes / (med * 1e-3) / 8e12);
  }
  return 0;
}
