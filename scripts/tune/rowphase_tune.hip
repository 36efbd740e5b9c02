// rowphase_tune.hip — does read/write phase separation also pay for 1-read +
// 1-write streams (a copy) and for the row-indexed gather / scatter-add?
// (tuning harness, not product code; it #includes the product kernels)
//
// Variants, interleaved rounds in one process, 4 GiB buffers, 8 M rows of 512 B
// with a random-permutation DoubleIndex:
//   copy mixed    : 16-B loads + stores, U = 4 strides (the bench's copy probe shape)
//   copy phased   : per block, a 64-KiB chunk read into LDS, then written
//   gather prod   : row_op_kernel<kAssignTo> (product)
//   gather phased : per block, 128 rows gathered into LDS, then written in order
//   add prod      : row_op_kernel<kAddFrom> (product)
//   add phased    : per block, 128 rows of x and of y read, summed into LDS, written to y
// Usage: rowphase_tune [rounds]
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

constexpr int kLdsF4 = 4096;  // 64 KiB per block

__global__ __launch_bounds__(kBlock) void copy_mixed(f4 *__restrict__ out, const f4 *__restrict__ in,
                                                     size_t n4) {
  const size_t stride = (size_t)gridDim.x * kBlock * 4;
  for (size_t i = (size_t)blockIdx.x * kBlock * 4 + threadIdx.x; i + 3 * kBlock < n4; i += stride) {
    f4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(in + i + u * kBlock);
#pragma unroll
    for (int u = 0; u < 4; ++u) out[i + u * kBlock] = v[u];
  }
}

// K chunks per launch; chunk = G blocks x kLdsF4 f4; block g takes 16-KiB tiles g, g+G, ...
template <int K>
__global__ __launch_bounds__(kBlock) void copy_phased(f4 *__restrict__ out, const f4 *__restrict__ in,
                                                      size_t n4, size_t chunk0) {
  constexpr int kTile = kBlock * 4, kTiles = kLdsF4 / kTile;
  __shared__ f4 res[kLdsF4];
  const size_t G = gridDim.x;
  for (int kc = 0; kc < K; ++kc) {
    const size_t lo = (chunk0 + kc) * G * kLdsF4;
    if (lo >= n4) return;
    for (int t = 0; t < kTiles; ++t) {
      const size_t tile0 = lo + ((size_t)t * G + blockIdx.x) * kTile;
      if (tile0 >= n4) break;
      f4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(in + tile0 + u * kBlock + threadIdx.x);
#pragma unroll
      for (int u = 0; u < 4; ++u) res[t * kTile + u * kBlock + threadIdx.x] = v[u];
    }
    __syncthreads();
    for (int t = 0; t < kTiles; ++t) {
      const size_t tile0 = lo + ((size_t)t * G + blockIdx.x) * kTile;
      if (tile0 >= n4) break;
#pragma unroll
      for (int u = 0; u < 4; ++u) out[tile0 + u * kBlock + threadIdx.x] = res[t * kTile + u * kBlock + threadIdx.x];
    }
    __syncthreads();
  }
}

// Rows of W = 128 floats (32 f4): a block's chunk is 128 consecutive index
// entries (rows); group of 32 lanes per row, 8 groups, 16 rows per group.
// ADD: y[id1] = y[id1] + x[id0]; else gather: y[id0] = x[id1].
template <bool ADD, int K>
__global__ __launch_bounds__(kBlock) void rows_phased(float *__restrict__ y, const float *__restrict__ x,
                                                      const gp_double_index *__restrict__ idx,
                                                      size_t n_rows, size_t chunk0) {
  constexpr int kVW = 32, kRows = kLdsF4 / kVW;  // 128 rows per block per chunk
  constexpr int kGroups = kBlock / kVW, kRowsPerGroup = kRows / kGroups;
  __shared__ f4 res[kLdsF4];
  const int lane = threadIdx.x % kVW, grp = threadIdx.x / kVW;
  f4 *yv = reinterpret_cast<f4 *>(y);
  const f4 *xv = reinterpret_cast<const f4 *>(x);
  const size_t G = gridDim.x;
  for (int kc = 0; kc < K; ++kc) {
    const size_t lo = ((chunk0 + kc) * G + blockIdx.x) * kRows;  // this block's first row
    if ((chunk0 + kc) * G * kRows >= n_rows) return;  // grid-uniform
    uint64_t src[kRowsPerGroup], dst[kRowsPerGroup];
#pragma unroll
    for (int i = 0; i < kRowsPerGroup; ++i) {  // all index entries first (independent loads)
      const size_t r = lo + (size_t)i * kGroups + grp;
      src[i] = dst[i] = ~0ull;
      if (r < n_rows) {
        const gp_double_index ix = idx[r];
        src[i] = ADD ? ix.id0 : ix.id1;
        dst[i] = ADD ? ix.id1 : ix.id0;
      }
    }
    f4 xs[kRowsPerGroup], ys[kRowsPerGroup];
#pragma unroll
    for (int i = 0; i < kRowsPerGroup; ++i)  // then every row load in flight
      if (src[i] != ~0ull) xs[i] = xv[src[i] * kVW + lane];
    if (ADD) {
#pragma unroll
      for (int i = 0; i < kRowsPerGroup; ++i)
        if (dst[i] != ~0ull) ys[i] = yv[dst[i] * kVW + lane];
    }
#pragma unroll
    for (int i = 0; i < kRowsPerGroup; ++i)
      if (src[i] != ~0ull) res[(i * kGroups + grp) * kVW + lane] = ADD ? ys[i] + xs[i] : xs[i];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kRowsPerGroup; ++i)
      if (dst[i] != ~0ull) yv[dst[i] * kVW + lane] = res[(i * kGroups + grp) * kVW + lane];
    __syncthreads();
  }
}

// Same, with the NEXT chunk's index entries loaded before this chunk's write
// phase, so each chunk waits for one round trip (the rows), not two.
template <bool ADD, int K>
__global__ __launch_bounds__(kBlock) void rows_phased_pf(float *__restrict__ y, const float *__restrict__ x,
                                                         const gp_double_index *__restrict__ idx,
                                                         size_t n_rows, size_t chunk0) {
  constexpr int kVW = 32, kRows = kLdsF4 / kVW;
  constexpr int kGroups = kBlock / kVW, kRowsPerGroup = kRows / kGroups;
  __shared__ f4 res[kLdsF4];
  const int lane = threadIdx.x % kVW, grp = threadIdx.x / kVW;
  f4 *yv = reinterpret_cast<f4 *>(y);
  const f4 *xv = reinterpret_cast<const f4 *>(x);
  const size_t G = gridDim.x;
  uint64_t src[kRowsPerGroup], dst[kRowsPerGroup];
  auto load_idx = [&](size_t c) {
    const size_t lo = (c * G + blockIdx.x) * kRows;
#pragma unroll
    for (int i = 0; i < kRowsPerGroup; ++i) {
      const size_t r = lo + (size_t)i * kGroups + grp;
      src[i] = dst[i] = ~0ull;
      if (r < n_rows) {
        const gp_double_index ix = idx[r];
        src[i] = ADD ? ix.id0 : ix.id1;
        dst[i] = ADD ? ix.id1 : ix.id0;
      }
    }
  };
  if (chunk0 * G * kRows >= n_rows) return;
  load_idx(chunk0);
  for (int kc = 0; kc < K; ++kc) {
    const size_t c = chunk0 + kc;
    if (c * G * kRows >= n_rows) return;  // grid-uniform
    f4 xs[kRowsPerGroup], ys[kRowsPerGroup];
#pragma unroll
    for (int i = 0; i < kRowsPerGroup; ++i)
      if (src[i] != ~0ull) xs[i] = xv[src[i] * kVW + lane];
    if (ADD) {
#pragma unroll
      for (int i = 0; i < kRowsPerGroup; ++i)
        if (dst[i] != ~0ull) ys[i] = yv[dst[i] * kVW + lane];
    }
#pragma unroll
    for (int i = 0; i < kRowsPerGroup; ++i)
      if (src[i] != ~0ull) res[(i * kGroups + grp) * kVW + lane] = ADD ? ys[i] + xs[i] : xs[i];
    uint64_t cur_dst[kRowsPerGroup];
#pragma unroll
    for (int i = 0; i < kRowsPerGroup; ++i) cur_dst[i] = dst[i];
    if (kc + 1 < K) load_idx(c + 1);  // prefetch: in flight during the write phase
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kRowsPerGroup; ++i)
      if (cur_dst[i] != ~0ull) yv[cur_dst[i] * kVW + lane] = res[(i * kGroups + grp) * kVW + lane];
    __syncthreads();
  }
}

template <bool ADD, int K>
void launch_rows_phased_pf(float *y, const float *x, const gp_double_index *idx, size_t n, int bpc) {
  const size_t G = (size_t)num_cus() * bpc, chunk = G * (kLdsF4 / 32);
  const size_t chunks = (n + chunk - 1) / chunk;
  for (size_t c = 0; c < chunks; c += K)
    hipLaunchKernelGGL((rows_phased_pf<ADD, K>), dim3((unsigned)G), dim3(kBlock), 0, 0, y, x, idx, n, c);
}

template <int K>
void launch_copy_phased(f4 *out, const f4 *in, size_t n4, int bpc) {
  const size_t G = (size_t)num_cus() * bpc, chunk = G * kLdsF4;
  const size_t chunks = (n4 + chunk - 1) / chunk;
  for (size_t c = 0; c < chunks; c += K)
    hipLaunchKernelGGL((copy_phased<K>), dim3((unsigned)G), dim3(kBlock), 0, 0, out, in, n4, c);
}

template <bool ADD, int K>
void launch_rows_phased(float *y, const float *x, const gp_double_index *idx, size_t n, int bpc) {
  const size_t G = (size_t)num_cus() * bpc, chunk = G * (kLdsF4 / 32);
  const size_t chunks = (n + chunk - 1) / chunk;
  for (size_t c = 0; c < chunks; c += K)
    hipLaunchKernelGGL((rows_phased<ADD, K>), dim3((unsigned)G), dim3(kBlock), 0, 0, y, x, idx, n, c);
}

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 5;
  const size_t bytes = 4ull << 30, n4 = bytes / 16, R = bytes / 512;
  float *x, *y, *y2;
  CK(hipMalloc(&x, bytes));
  CK(hipMalloc(&y, bytes));
  CK(hipMalloc(&y2, bytes));
  CK(hipMemset(y, 0, bytes));
  std::vector<float> hx(1 << 24);
  for (size_t i = 0; i < hx.size(); ++i) hx[i] = (float)(i % 977) * 0.25f;
  for (size_t off = 0; off < bytes / 4; off += hx.size())
    CK(hipMemcpy(x + off, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
  std::vector<uint64_t> perm(R);
  std::iota(perm.begin(), perm.end(), 0);
  std::mt19937_64 rng(5);
  std::shuffle(perm.begin(), perm.end(), rng);
  std::vector<gp_double_index> h(R);
  for (size_t r = 0; r < R; ++r) h[r] = gp_double_index{r, perm[r]};
  gp_double_index *idx;
  CK(hipMalloc(&idx, R * sizeof(gp_double_index)));
  CK(hipMemcpy(idx, h.data(), R * sizeof(gp_double_index), hipMemcpyHostToDevice));

  // correctness: phased gather / add == product on the same inputs
  {
    size_t bad = 0;
    std::vector<float> a(1 << 22), b(1 << 22);
    CK(hipMemset(y, 0, bytes));
    CK(hipMemset(y2, 0, bytes));
    gp_gather_rows(y, x, idx, R, {0, 0}, 128, (size_t)-1, nullptr);
    launch_rows_phased_pf<false, 8>(y2, x, idx, R, 2);
    gp_scatter_add_rows(y, x, idx, R, {0, 0}, 128, (size_t)-1, nullptr);
    launch_rows_phased_pf<true, 8>(y2, x, idx, R, 2);
    CK(hipDeviceSynchronize());
    for (size_t off = 0; off < bytes / 4; off += bytes / 4 / 8) {
      CK(hipMemcpy(a.data(), y + off, a.size() * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(b.data(), y2 + off, b.size() * 4, hipMemcpyDeviceToHost));
      for (size_t i = 0; i < a.size(); ++i) bad += std::memcmp(&a[i], &b[i], 4) != 0;
    }
    std::printf("phased gather+add vs product, sampled 32 Mi floats: %zu mismatches\n", bad);
  }

  struct V {
    std::string name;
    double bytes;
    std::function<void()> run;
    std::vector<float> ms;
  };
  std::vector<V> vs;
  const unsigned G8 = num_cus() * 8;
  f4 *xv = reinterpret_cast<f4 *>(x), *yv = reinterpret_cast<f4 *>(y);
  const double gat_b = 2.0 * bytes + 16.0 * R, add_b = 3.0 * bytes + 16.0 * R;
  vs.push_back(V{"copy mixed", 2.0 * bytes, [=]() { copy_mixed<<<G8, kBlock>>>(yv, xv, n4); }, {}});
  vs.push_back(V{"copy phased k4 bpc2", 2.0 * bytes, [=]() { launch_copy_phased<4>(yv, xv, n4, 2); }, {}});
  vs.push_back(V{"copy phased k8 bpc2", 2.0 * bytes, [=]() { launch_copy_phased<8>(yv, xv, n4, 2); }, {}});
  vs.push_back(V{"gather prod", gat_b, [=]() { gp_gather_rows(y, x, idx, R, {0, 0}, 128, (size_t)-1, nullptr); }, {}});
  vs.push_back(V{"gather phased k4 bpc2", gat_b, [=]() { launch_rows_phased<false, 4>(y, x, idx, R, 2); }, {}});
  vs.push_back(V{"gather phased k8 bpc2", gat_b, [=]() { launch_rows_phased<false, 8>(y, x, idx, R, 2); }, {}});
  vs.push_back(V{"gather phased-pf k8 bpc2", gat_b, [=]() { launch_rows_phased_pf<false, 8>(y, x, idx, R, 2); }, {}});
  vs.push_back(V{"gather phased-pf k16 bpc2", gat_b, [=]() { launch_rows_phased_pf<false, 16>(y, x, idx, R, 2); }, {}});
  vs.push_back(V{"gather phased-pf k8 bpc4", gat_b, [=]() { launch_rows_phased_pf<false, 8>(y, x, idx, R, 4); }, {}});
  vs.push_back(V{"add prod", add_b, [=]() { gp_scatter_add_rows(y, x, idx, R, {0, 0}, 128, (size_t)-1, nullptr); }, {}});
  vs.push_back(V{"add phased k4 bpc2", add_b, [=]() { launch_rows_phased<true, 4>(y, x, idx, R, 2); }, {}});
  vs.push_back(V{"add phased k8 bpc2", add_b, [=]() { launch_rows_phased<true, 8>(y, x, idx, R, 2); }, {}});
  vs.push_back(V{"add phased-pf k8 bpc2", add_b, [=]() { launch_rows_phased_pf<true, 8>(y, x, idx, R, 2); }, {}});
  vs.push_back(V{"add phased-pf k16 bpc2", add_b, [=]() { launch_rows_phased_pf<true, 16>(y, x, idx, R, 2); }, {}});

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
    std::printf("%-26s %10.4f %10.4f %10.1f %8.4f\n", v.name.c_str(), med, v.ms[0], gbs, gbs / 8000.0);
  }
  return 0;
}
