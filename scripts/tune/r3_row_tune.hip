// r3_row_tune.hip — round-3 probe for the unplanned row ops (tuning harness,
// not product code; it #includes the product kernels).
//
// Questions (8 M rows of 128 floats, 4 GiB x / y, random-permutation and
// identity DoubleIndex):
//  1. How much destination locality does the op-order random scatter-add
//     need?  The destination-sorted plan residual runs ~78 % of 8 TB/s
//     through row_wave_kernel, the op-order index ~64 % through row_op_kernel.
//     Here: the index binned by destination row >> s (order inside a bin
//     random, as a device counting sort leaves it), s = 6..18, through the
//     sorted (wave-map) path.
//  2. What does a device counting sort by destination bin cost (histogram,
//     scan, scatter)?  And a device index scan (dense-tile flags) + D2H + sync?
//  3. An indexed sweep (row_sweep_kernel): the bucket-sum sweep's chunk scheme
//     (read phase into LDS + registers, then a write phase) with per-row
//     addresses from the chunk's index entries staged in LDS.  On an identity
//     index it is the 1-bucket sweep plus 16 B of index per row; on a sorted
//     residual the write phase is a front-to-back walk.
// Every variant is checked bit for bit against the production kernels.
// Usage: r3_row_tune [rounds]
#include "../../geeps_amd/csrc/gp_reduce.hip"

#include <algorithm>
#include <chrono>
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
constexpr uint64_t kDead = ~0ull;

// ---------------------------------------------------------------------------
// indexed sweep: OP kAddFrom (y[to] += x[from]), kInitFrom (y[to] = 0 + x[from]),
// kAssignTo (y[to] = x[from], from = id1, to = id0).  128-float rows, no limit.
// ---------------------------------------------------------------------------
template <int OP, int RT, int TG, int U, int KL>
__global__ __launch_bounds__(kBlock) void row_sweep_kernel(float *__restrict__ y, const float *__restrict__ x,
                                                           const gp_double_index *__restrict__ index,
                                                           size_t n_rows, uint64_t off0, uint64_t off1,
                                                           size_t chunk) {
  constexpr int kVW = 32;
  constexpr int kTile = kBlock * U;
  constexpr int kTR = kTile / kVW;  // rows per tile
  constexpr int kT = KL + RT;
  static_assert(kT % TG == 0, "whole bursts");
  constexpr int kE = kT * kTR;
  constexpr int S = OP == kAddFrom ? 2 : 1;
  __shared__ f4 res[KL > 0 ? KL * kTile : 1];
  __shared__ uint64_t efrom[kE], eto[kE];
  f4 keep[RT][U];
  const size_t G = gridDim.x;
  const size_t tile0 = chunk * G * kT;
  if (tile0 * kTR >= n_rows) return;
  for (int q = threadIdx.x; q < kE; q += kBlock) {
    const int t = q / kTR, j = q % kTR;
    const size_t e = (tile0 + (size_t)t * G + blockIdx.x) * kTR + j;
    uint64_t from = kDead, to = kDead;
    if (e < n_rows) row_endpoints<OP>(index[e], off0, off1, from, to);
    efrom[q] = from;
    eto[q] = to;
  }
  __syncthreads();
  typedef __attribute__((address_space(1))) f4 GF4;
  const int col = threadIdx.x % kVW, rw = threadIdx.x / kVW;
  const GF4 *yv = reinterpret_cast<const GF4 *>(reinterpret_cast<uintptr_t>(y));
  const GF4 *xv = reinterpret_cast<const GF4 *>(reinterpret_cast<uintptr_t>(x));
#pragma unroll
  for (int k = 0; k < S; ++k) {
    const bool ystream = OP == kAddFrom && k == 0;
#pragma unroll
    for (int t0 = 0; t0 < kT; t0 += TG) {
      f4 v[TG][U];
#pragma unroll
      for (int j = 0; j < TG; ++j)
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int e = (t0 + j) * kTR + rw + 8 * u;
          const uint64_t row = ystream ? eto[e] : efrom[e];
          v[j][u] = f4(0.0f);
          if (row != kDead) v[j][u] = __builtin_nontemporal_load((ystream ? yv : xv) + row * kVW + col);
        }
#pragma unroll
      for (int j = 0; j < TG; ++j) {
        const int t = t0 + j;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const f4 first = OP == kInitFrom ? f4(0.0f) + v[j][u] : v[j][u];
          if (t < KL) {
            f4 &r = res[t * kTile + u * kBlock + threadIdx.x];
            r = k == 0 ? first : r + v[j][u];
          } else {
            f4 &r = keep[t >= KL ? t - KL : 0][u];
            r = k == 0 ? first : r + v[j][u];
          }
        }
      }
    }
  }
  __syncthreads();
  GF4 *yo = reinterpret_cast<GF4 *>(reinterpret_cast<uintptr_t>(y));
#pragma unroll
  for (int t = 0; t < kT; ++t)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = t * kTR + rw + 8 * u;
      const uint64_t to = eto[e];
      if (to != kDead)
        __builtin_nontemporal_store(t < KL ? res[t * kTile + u * kBlock + threadIdx.x]
                                           : keep[t >= KL ? t - KL : 0][u],
                                    yo + to * kVW + col);
    }
}

template <int OP, int RT, int TG, int U, int KL>
void launch_sweep(float *y, const float *x, const gp_double_index *ix, size_t n) {
  const size_t G = (size_t)num_cus();
  const size_t rows_per_chunk = G * (KL + RT) * (kBlock * U / 32);
  const size_t chunks = (n + rows_per_chunk - 1) / rows_per_chunk;
  for (size_t c = 0; c < chunks; ++c)
    hipLaunchKernelGGL((row_sweep_kernel<OP, RT, TG, U, KL>), dim3((unsigned)G), dim3(kBlock), 0, 0, y, x,
                       ix, n, 0, 0, c);
}

// ---------------------------------------------------------------------------
// device counting sort of a DoubleIndex by destination row >> s
// ---------------------------------------------------------------------------
constexpr int kHistLds = 16384;

__global__ __launch_bounds__(kBlock) void bin_hist_kernel(const gp_double_index *__restrict__ idx, size_t n,
                                                          int s, uint32_t nbins, uint32_t *hist,
                                                          size_t per_block) {
  __shared__ uint32_t h[kHistLds];
  const bool lds = nbins <= kHistLds;
  if (lds)
    for (uint32_t b = threadIdx.x; b < nbins; b += kBlock) h[b] = 0;
  __syncthreads();
  const size_t lo = blockIdx.x * per_block, hi = lo + per_block < n ? lo + per_block : n;
  for (size_t e = lo + threadIdx.x; e < hi; e += kBlock) {
    const uint32_t b = (uint32_t)(idx[e].id1 >> s);
    if (lds)
      atomicAdd(&h[b], 1u);
    else
      atomicAdd(&hist[b], 1u);
  }
  __syncthreads();
  if (lds)
    for (uint32_t b = threadIdx.x; b < nbins; b += kBlock)
      if (h[b]) atomicAdd(&hist[b], h[b]);
}

// one block: exclusive scan of hist into cursor
__global__ __launch_bounds__(1024) void bin_scan_kernel(const uint32_t *hist, uint32_t nbins, uint32_t *cursor) {
  __shared__ uint32_t part[1024];
  const uint32_t per = (nbins + 1023) / 1024;
  const uint32_t lo = threadIdx.x * per, hi = min(lo + per, nbins);
  uint32_t s = 0;
  for (uint32_t b = lo; b < hi; ++b) s += hist[b];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const uint32_t v = threadIdx.x >= (unsigned)off ? part[threadIdx.x - off] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  uint32_t run = threadIdx.x ? part[threadIdx.x - 1] : 0;
  for (uint32_t b = lo; b < hi; ++b) {
    cursor[b] = run;
    run += hist[b];
  }
}

__global__ __launch_bounds__(kBlock) void bin_scatter_kernel(const gp_double_index *__restrict__ idx, size_t n,
                                                             int s, uint32_t nbins, uint32_t *cursor,
                                                             gp_double_index *__restrict__ out,
                                                             size_t per_block) {
  __shared__ uint32_t h[kHistLds];
  __shared__ uint32_t base[kHistLds];
  const bool lds = nbins <= kHistLds;
  const size_t lo = blockIdx.x * per_block, hi = lo + per_block < n ? lo + per_block : n;
  if (lds) {
    for (uint32_t b = threadIdx.x; b < nbins; b += kBlock) h[b] = 0;
    __syncthreads();
    for (size_t e = lo + threadIdx.x; e < hi; e += kBlock) atomicAdd(&h[(uint32_t)(idx[e].id1 >> s)], 1u);
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nbins; b += kBlock) {
      base[b] = h[b] ? atomicAdd(&cursor[b], h[b]) : 0;
      h[b] = 0;
    }
    __syncthreads();
  }
  for (size_t e = lo + threadIdx.x; e < hi; e += kBlock) {
    const gp_double_index ix = idx[e];
    const uint32_t b = (uint32_t)(ix.id1 >> s);
    const uint32_t pos = lds ? base[b] + atomicAdd(&h[b], 1u) : atomicAdd(&cursor[b], 1u);
    out[pos] = ix;
  }
}

// ---------------------------------------------------------------------------
// index scan: per 64-entry tile, bit 0 = dense (id0 and id1 step by one inside
// the tile, every entry live), bit 1 = continues the previous tile's last entry
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void index_scan_kernel(const gp_double_index *__restrict__ idx, size_t n,
                                                            uint8_t *flags, unsigned long long *max_dst) {
  const int wl = threadIdx.x & 63;
  const size_t tiles = (n + 63) / 64;
  const size_t wave = ((size_t)blockIdx.x * kBlock + threadIdx.x) / 64;
  const size_t wstride = (size_t)gridDim.x * (kBlock / 64);
  unsigned long long mx = 0;
  for (size_t t = wave; t < tiles; t += wstride) {
    const size_t e = t * 64 + wl;
    const bool live = e < n;
    gp_double_index ix = {0, 0}, pv = {0, 0};
    if (live) ix = idx[e];
    if (wl == 0 && e > 0) pv = idx[e - 1];
    const uint64_t p0 = shfl64(ix.id0, (wl + 63) & 63), p1 = shfl64(ix.id1, (wl + 63) & 63);
    bool step = wl == 0 ? true : (ix.id0 == p0 + 1 && ix.id1 == p1 + 1);
    const bool cont = e > 0 && ix.id0 == pv.id0 + 1 && ix.id1 == pv.id1 + 1;
    const bool dense = __all(live && step);
    const bool c0 = __shfl(cont ? 1 : 0, 0, 64);
    if (live && ix.id1 > mx) mx = ix.id1;
    if (wl == 0) flags[t] = (dense ? 1 : 0) | (c0 ? 2 : 0);
  }
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long o2 = shfl64(mx, (wl + o) & 63);
    mx = o2 > mx ? o2 : mx;
  }
  if (wl == 0) atomicMax(max_dst, mx);
}

__global__ void mismatch_kernel(const uint32_t *a, const uint32_t *b, size_t n, unsigned long long *cnt) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  unsigned long long c = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) c += a[i] != b[i];
  if (c) atomicAdd(cnt, c);
}

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 5;
  float *x, *y, *y0, *yr;
  CK(hipMalloc(&x, N * 4));
  CK(hipMalloc(&y, N * 4));
  CK(hipMalloc(&y0, N * 4));
  CK(hipMalloc(&yr, N * 4));
  std::mt19937_64 g(3);
  std::vector<uint64_t> perm(R);
  std::iota(perm.begin(), perm.end(), 0);
  std::shuffle(perm.begin(), perm.end(), g);
  {
    std::vector<float> h(N);
    std::uniform_real_distribution<float> d(-0.5f, 0.5f);
    for (size_t i = 0; i < N; i += 1) h[i] = d(g);
    CK(hipMemcpy(x, h.data(), N * 4, hipMemcpyHostToDevice));
    for (size_t i = 0; i < N; i += 1) h[i] = d(g);
    CK(hipMemcpy(y0, h.data(), N * 4, hipMemcpyHostToDevice));
  }
  auto upload = [&](const std::vector<gp_double_index> &v) {
    gp_double_index *p;
    CK(hipMalloc(&p, R * 16));
    CK(hipMemcpy(p, v.data(), R * 16, hipMemcpyHostToDevice));
    return p;
  };
  std::vector<gp_double_index> a(R), b(R), c(R);
  for (size_t r = 0; r < R; ++r) {
    a[r] = {r, perm[r]};
    b[perm[r]] = {r, perm[r]};
    c[r] = {r, r};
  }
  gp_double_index *rnd = upload(a), *srt = upload(b), *idn = upload(c);
  // gather index: destination id0 in order, source id1 random (what a gather
  // plan's residual and the reference's Read index hold)
  const int bins[] = {6, 9, 12, 15, 18};
  std::vector<gp_double_index *> binned;
  for (int s : bins) {
    std::vector<gp_double_index> v = a;
    std::stable_sort(v.begin(), v.end(),
                     [s](const gp_double_index &p, const gp_double_index &q) { return (p.id1 >> s) < (q.id1 >> s); });
    binned.push_back(upload(v));
  }
  gp_double_index *dbin;
  CK(hipMalloc(&dbin, R * 16));
  uint32_t *hist, *cursor;
  CK(hipMalloc(&hist, (1u << 20) * 4));
  CK(hipMalloc(&cursor, (1u << 20) * 4));
  uint8_t *flags, *hflags;
  unsigned long long *maxd, *cnt;
  CK(hipMalloc(&flags, R / 64 + 64));
  CK(hipHostMalloc(&hflags, R / 64 + 64, hipHostMallocDefault));
  CK(hipMalloc(&maxd, 8));
  CK(hipMalloc(&cnt, 8));

  const size_t G = (size_t)num_cus();
  auto reset = [&] { CK(hipMemcpyAsync(y, y0, N * 4, hipMemcpyDeviceToDevice, 0)); };
  auto prod_add = [&](const gp_double_index *ix, bool sorted) {
    return [=] { launch_row_op<kAddFrom>(y, x, ix, R, {0, 0}, W, ~size_t(0), 0, sorted); };
  };
  auto prod_init = [&](const gp_double_index *ix, bool sorted) {
    return [=] { launch_row_op<kInitFrom>(y, x, ix, R, {0, 0}, W, ~size_t(0), 0, sorted); };
  };
  auto prod_gather = [&](const gp_double_index *ix) {
    return [=] { launch_row_op<kAssignTo>(y, x, ix, R, {0, 0}, W, ~size_t(0), 0, true); };
  };
  auto dev_bin = [&](int s, int part) {  // part: 1 hist, 2 +scan, 3 +scatter
    return [=] {
      const uint32_t nbins = (uint32_t)((R + (1ull << s) - 1) >> s);
      const size_t nb = 4 * G, per = (R + nb - 1) / nb;
      CK(hipMemsetAsync(hist, 0, nbins * 4, 0));
      hipLaunchKernelGGL(bin_hist_kernel, dim3((unsigned)nb), dim3(kBlock), 0, 0, rnd, R, s, nbins, hist, per);
      if (part >= 2) hipLaunchKernelGGL(bin_scan_kernel, dim3(1), dim3(1024), 0, 0, hist, nbins, cursor);
      if (part >= 3)
        hipLaunchKernelGGL(bin_scatter_kernel, dim3((unsigned)nb), dim3(kBlock), 0, 0, rnd, R, s, nbins, cursor,
                           dbin, per);
    };
  };
  auto scan = [&](bool d2h) {
    return [=] {
      CK(hipMemsetAsync(maxd, 0, 8, 0));
      hipLaunchKernelGGL(index_scan_kernel, dim3((unsigned)(G * 4)), dim3(kBlock), 0, 0, rnd, R, flags, maxd);
      if (d2h) {
        CK(hipMemcpyAsync(hflags, flags, R / 64, hipMemcpyDeviceToHost, 0));
        CK(hipStreamSynchronize(0));
      }
    };
  };

  const double add_b = 3.0 * N * 4 + 16.0 * R, one_b = 2.0 * N * 4 + 16.0 * R;
  struct V {
    std::string name;
    std::function<void()> f;
    double bytes;
    int check;  // 0 none, 1 add vs yr(add), 2 init, 3 gather
    const gp_double_index *ref_ix;
  };
  std::vector<V> vs = {
      {"add  rand  row_op (prod)", prod_add(rnd, false), add_b, 0, nullptr},
      {"add  ident row_op (prod)", prod_add(idn, false), add_b, 0, nullptr},
      {"add  sorted wave (prod plan)", prod_add(srt, true), add_b, 1, srt},
  };
  for (size_t i = 0; i < binned.size(); ++i)
    vs.push_back({"add  bin" + std::to_string(bins[i]) + " wave", prod_add(binned[i], true), add_b, 1, binned[i]});
  vs.push_back({"add  ident dense sweep (plan)", [&] {
                  BucketPtrs bp = {};
                  bp.p[0] = x;
                  launch_bucket_sum_nb<1>(y, y, bp, N, 0);
                },
                3.0 * N * 4, 0, nullptr});
  vs.push_back({"add  ident rsweep 15/8/4/9", [&] { launch_sweep<kAddFrom, 15, 8, 4, 9>(y, x, idn, R); }, add_b, 1, idn});
  vs.push_back({"add  ident rsweep 15/2/4/9", [&] { launch_sweep<kAddFrom, 15, 2, 4, 9>(y, x, idn, R); }, add_b, 1, idn});
  vs.push_back({"add  ident rsweep 7/1/8/4", [&] { launch_sweep<kAddFrom, 7, 1, 8, 4>(y, x, idn, R); }, add_b, 1, idn});
  vs.push_back({"add  sorted rsweep 15/8/4/9", [&] { launch_sweep<kAddFrom, 15, 8, 4, 9>(y, x, srt, R); }, add_b, 1, srt});
  vs.push_back({"add  sorted rsweep 7/1/8/4", [&] { launch_sweep<kAddFrom, 7, 1, 8, 4>(y, x, srt, R); }, add_b, 1, srt});
  vs.push_back({"add  bin12 rsweep 15/8/4/9", [&] { launch_sweep<kAddFrom, 15, 8, 4, 9>(y, x, binned[2], R); }, add_b, 1, binned[2]});
  vs.push_back({"add  rand  rsweep 15/8/4/9", [&] { launch_sweep<kAddFrom, 15, 8, 4, 9>(y, x, rnd, R); }, add_b, 1, rnd});
  vs.push_back({"init rand  wave (prod)", prod_init(rnd, false), one_b, 0, nullptr});
  vs.push_back({"init ident wave (prod)", prod_init(idn, false), one_b, 0, nullptr});
  vs.push_back({"init sorted wave (prod plan)", prod_init(srt, true), one_b, 2, srt});
  vs.push_back({"init bin12 wave", prod_init(binned[2], true), one_b, 2, binned[2]});
  vs.push_back({"init ident rsweep 15/8/4/9", [&] { launch_sweep<kInitFrom, 15, 8, 4, 9>(y, x, idn, R); }, one_b, 2, idn});
  vs.push_back({"init sorted rsweep 15/8/4/9", [&] { launch_sweep<kInitFrom, 15, 8, 4, 9>(y, x, srt, R); }, one_b, 2, srt});
  vs.push_back({"init sorted rsweep 15/4/4/9", [&] { launch_sweep<kInitFrom, 15, 4, 4, 9>(y, x, srt, R); }, one_b, 2, srt});
  vs.push_back({"init sorted rsweep 7/4/4/9", [&] { launch_sweep<kInitFrom, 7, 4, 4, 9>(y, x, srt, R); }, one_b, 2, srt});
  vs.push_back({"gath rand  wave (prod plan)", prod_gather(rnd), one_b, 3, rnd});
  vs.push_back({"gath rand  rsweep 15/8/4/9", [&] { launch_sweep<kAssignTo, 15, 8, 4, 9>(y, x, rnd, R); }, one_b, 3, rnd});
  vs.push_back({"gath rand  rsweep 7/4/4/9", [&] { launch_sweep<kAssignTo, 7, 4, 4, 9>(y, x, rnd, R); }, one_b, 3, rnd});
  vs.push_back({"gath ident rsweep 15/8/4/9", [&] { launch_sweep<kAssignTo, 15, 8, 4, 9>(y, x, idn, R); }, one_b, 3, idn});
  for (int s : {10, 12, 14, 16}) {
    vs.push_back({"devbin s" + std::to_string(s) + " hist", dev_bin(s, 1), 16.0 * R, 0, nullptr});
    vs.push_back({"devbin s" + std::to_string(s) + " all", dev_bin(s, 3), 48.0 * R, 0, nullptr});
  }
  vs.push_back({"index scan", scan(false), 16.0 * R, 0, nullptr});
  vs.push_back({"index scan + D2H + sync", scan(true), 16.0 * R, 0, nullptr});

  // ---- checks: each variant once from y0, against the production kernel
  // (add: row_op_kernel on the same index; init / gather likewise)
  auto check = [&](const V &v) {
    reset();
    if (v.check == 1)
      launch_row_op<kAddFrom>(y, x, v.ref_ix, R, {0, 0}, W, ~size_t(0), 0, false);
    else if (v.check == 2)
      launch_row_op<kInitFrom>(y, x, v.ref_ix, R, {0, 0}, W, ~size_t(0), 0, false);
    else
      launch_row_op<kAssignTo>(y, x, v.ref_ix, R, {0, 0}, W, ~size_t(0), 0, false);
    CK(hipMemcpyAsync(yr, y, N * 4, hipMemcpyDeviceToDevice, 0));
    reset();
    v.f();
    CK(hipMemsetAsync(cnt, 0, 8, 0));
    hipLaunchKernelGGL(mismatch_kernel, dim3(1024), dim3(256), 0, 0, (const uint32_t *)y, (const uint32_t *)yr, N,
                       cnt);
    unsigned long long h = 0;
    CK(hipMemcpy(&h, cnt, 8, hipMemcpyDeviceToHost));
    return h;
  };
  for (auto &v : vs)
    if (v.check) {
      const unsigned long long m = check(v);
      std::printf("check %-32s mismatches %llu\n", v.name.c_str(), m);
      if (m) return 3;
    }
  {  // device binning: a permutation of the entries, bins ascending
    dev_bin(12, 3)();
    std::vector<gp_double_index> h(R);
    CK(hipMemcpy(h.data(), dbin, R * 16, hipMemcpyDeviceToHost));
    bool ok = true;
    std::vector<uint8_t> seen(R, 0);
    for (size_t r = 0; r < R && ok; ++r) {
      ok = h[r].id0 < R && !seen[h[r].id0] && h[r].id1 == perm[h[r].id0] && (r == 0 || (h[r - 1].id1 >> 12) <= (h[r].id1 >> 12));
      if (ok) seen[h[r].id0] = 1;
    }
    std::printf("check devbin s12 %s\n", ok ? "ok" : "FAILED");
    scan(true)();
    unsigned long long m = 0;
    CK(hipMemcpy(&m, maxd, 8, hipMemcpyDeviceToHost));
    std::printf("check index scan max %llu (expect %zu) flags[0..3] %d %d %d %d\n", m, R - 1, hflags[0], hflags[1],
                hflags[2], hflags[3]);
    if (!ok) return 3;
  }
  reset();
  CK(hipDeviceSynchronize());

  hipEvent_t ea, eb;
  CK(hipEventCreate(&ea));
  CK(hipEventCreate(&eb));
  std::vector<std::vector<float>> ms(vs.size());
  std::vector<std::vector<double>> wall(vs.size());
  for (auto &v : vs) v.f();
  CK(hipDeviceSynchronize());
  for (int r = 0; r < rounds; ++r) {
    for (size_t i = 0; i < vs.size(); ++i) {
      CK(hipDeviceSynchronize());
      const auto t0 = std::chrono::steady_clock::now();
      CK(hipEventRecord(ea, 0));
      vs[i].f();
      CK(hipEventRecord(eb, 0));
      CK(hipEventSynchronize(eb));
      const auto t1 = std::chrono::steady_clock::now();
      float t = 0;
      CK(hipEventElapsedTime(&t, ea, eb));
      ms[i].push_back(t);
      wall[i].push_back(std::chrono::duration<double, std::milli>(t1 - t0).count());
    }
    std::fprintf(stderr, "round %d done\n", r);
  }
  CK(hipGetLastError());
  std::printf("%-34s %9s %9s %9s %8s %9s\n", "variant", "med_ms", "min_ms", "TB/s", "%8TB/s", "wall_ms");
  for (size_t i = 0; i < vs.size(); ++i) {
    auto m = ms[i];
    auto w = wall[i];
    std::sort(m.begin(), m.end());
    std::sort(w.begin(), w.end());
    const double med = m[m.size() / 2];
    const double tbs = vs[i].bytes / (med * 1e-3) / 1e12;
    std::printf("%-34s %9.4f %9.4f %9.3f %7.1f%% %9.4f\n", vs[i].name.c_str(), med, m[0], tbs, 100.0 * tbs / 8.0,
                w[w.size() / 2]);
  }
  return 0;
}
