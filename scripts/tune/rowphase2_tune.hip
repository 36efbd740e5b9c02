// rowphase2_tune.hip — phase-separated row ops with the index off the critical
// path (tuning harness, not product code; it #includes the product kernels).
//
// rowphase_tune.hip found a phased gather / scatter-add slower than the mixed
// production kernel at 64 KiB of LDS per block: every chunk paid the index
// round trip, then the row round trip.  Here a block owns ROWS consecutive
// index entries per chunk (RowData rows of 128 floats, 32 lanes per row), keeps
// the chunk's endpoints in LDS (double-buffered) and loads the NEXT chunk's
// entries while this chunk's rows are read, so each phase waits only for rows.
// Read phase: S rows per 32-lane group in flight per sub-batch, results parked
// in LDS.  Write phase: the rows go out.  Variants over ROWS (LDS), S, block
// size and chunks per launch K; 4 GiB tables, 8 M rows, random permutation.
// Usage: rowphase2_tune [rounds]
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

constexpr int kVW = 32;  // f4 per 128-float row

template <int OP, int BS, int ROWS, int S>
__global__ __launch_bounds__(BS) void rows_ph2(float *__restrict__ y, const float *__restrict__ x,
                                               const gp_double_index *__restrict__ idx,
                                               size_t n_rows, uint64_t off0, uint64_t off1,
                                               size_t limit, size_t chunk0, int K) {
  constexpr int kGroups = BS / kVW;
  constexpr int kPerGroup = ROWS / kGroups;  // rows per group per chunk
  static_assert(ROWS % kGroups == 0 && kPerGroup % S == 0, "shape");
  constexpr int kIdxPerThread = (ROWS + BS - 1) / BS;
  __shared__ f4 res[ROWS * kVW];
  __shared__ uint64_t efrom[2][ROWS], eto[2][ROWS];
  const int lane = threadIdx.x % kVW, grp = threadIdx.x / kVW;
  const size_t G = gridDim.x;
  f4 *yv = reinterpret_cast<f4 *>(y);
  const f4 *xv = reinterpret_cast<const f4 *>(x);
  constexpr uint64_t kNone = ~0ull;

  gp_double_index pre[kIdxPerThread];
  auto load_idx = [&](size_t c) {
    const size_t lo = (c * G + blockIdx.x) * ROWS;
#pragma unroll
    for (int i = 0; i < kIdxPerThread; ++i) {
      const size_t e = (size_t)i * BS + threadIdx.x;
      pre[i].id0 = pre[i].id1 = kNone;
      if (e < ROWS && lo + e < n_rows) pre[i] = idx[lo + e];
    }
  };
  auto park_idx = [&](int buf) {
#pragma unroll
    for (int i = 0; i < kIdxPerThread; ++i) {
      const int e = i * BS + threadIdx.x;
      if (e < ROWS) {
        uint64_t from = kNone, to = kNone;
        if (pre[i].id0 != kNone || pre[i].id1 != kNone) row_endpoints<OP>(pre[i], off0, off1, from, to);
        efrom[buf][e] = from;
        eto[buf][e] = to;
      }
    }
  };
  if (chunk0 * G * ROWS >= n_rows) return;
  load_idx(chunk0);
  park_idx(0);
  __syncthreads();
  int buf = 0;
  for (int kc = 0; kc < K; ++kc) {
    const size_t c = chunk0 + kc;
    if (c * G * ROWS >= n_rows) return;  // grid-uniform
    const bool more = kc + 1 < K && (c + 1) * G * ROWS < n_rows;
    if (more) load_idx(c + 1);  // in flight during the read phase
    // read phase
#pragma unroll 1
    for (int sb = 0; sb < kPerGroup / S; ++sb) {
      f4 xs[S], ys[S];
      uint64_t fr[S], to[S];
      bool whole[S];
#pragma unroll
      for (int i = 0; i < S; ++i) {
        const int r = (sb * S + i) * kGroups + grp;
        fr[i] = efrom[buf][r];
        to[i] = eto[buf][r];
        const uint64_t guarded = (OP == kAssignTo) ? to[i] : fr[i];
        whole[i] = fr[i] != kNone && (guarded + 1) * (kVW * 4) <= limit;
      }
#pragma unroll
      for (int i = 0; i < S; ++i)
        if (whole[i]) xs[i] = __builtin_nontemporal_load(xv + fr[i] * kVW + lane);
      if (OP == kAddFrom) {
#pragma unroll
        for (int i = 0; i < S; ++i)
          if (whole[i]) ys[i] = yv[to[i] * kVW + lane];
      }
#pragma unroll
      for (int i = 0; i < S; ++i) {
        const int r = (sb * S + i) * kGroups + grp;
        if (whole[i])
          res[r * kVW + lane] = OP == kAddFrom ? ys[i] + xs[i] : (OP == kInitFrom ? f4(0.0f) + xs[i] : xs[i]);
      }
    }
    if (more) park_idx(buf ^ 1);  // the previous chunk's buffer: free since its write phase
    __syncthreads();
    // write phase
#pragma unroll 4
    for (int i = 0; i < kPerGroup; ++i) {
      const int r = i * kGroups + grp;
      const uint64_t fr = efrom[buf][r], to = eto[buf][r];
      if (fr == kNone) continue;
      const uint64_t guarded = (OP == kAssignTo) ? to : fr;
      if ((guarded + 1) * (kVW * 4) <= limit) {
        yv[to * kVW + lane] = res[r * kVW + lane];
      } else {  // straddles num_vals_limit: element-wise guard, straight from x
        for (int e = lane; e < kVW * 4; e += kVW) {
          if (guarded * (kVW * 4) + e < limit) {
            const float v = x[fr * (kVW * 4) + e];
            if (OP == kAddFrom) y[to * (kVW * 4) + e] += v;
            else if (OP == kInitFrom) y[to * (kVW * 4) + e] = 0.0f + v;
            else y[to * (kVW * 4) + e] = v;
          } else if (OP == kInitFrom) {
            y[to * (kVW * 4) + e] = 0.0f;
          }
        }
      }
    }
    __syncthreads();
    buf ^= 1;
  }
}

template <int OP, int BS, int ROWS, int S>
void launch_ph2(float *y, const float *x, const gp_double_index *idx, size_t n, int K) {
  const size_t G = (size_t)num_cus(), chunk = G * ROWS;
  const size_t chunks = (n + chunk - 1) / chunk;
  for (size_t c = 0; c < chunks; c += K)
    hipLaunchKernelGGL((rows_ph2<OP, BS, ROWS, S>), dim3((unsigned)G), dim3(BS), 0, 0, y, x, idx, n,
                       (uint64_t)0, (uint64_t)0, (size_t)-1, c, K);
}

// copy, phased at 160 KiB per block (1 block per CU), for the ceiling
template <int K>
__global__ __launch_bounds__(kBlock) void copy_ph160(f4 *__restrict__ out, const f4 *__restrict__ in,
                                                     size_t n4, size_t chunk0) {
  constexpr int kLds = 10240, kTile = kBlock * 4, kTiles = kLds / kTile;
  __shared__ f4 res[kLds];
  const size_t G = gridDim.x;
  for (int kc = 0; kc < K; ++kc) {
    const size_t lo = (chunk0 + kc) * G * kLds;
    if (lo >= n4) return;
    for (int t = 0; t < kTiles; ++t) {
      const size_t tile0 = lo + ((size_t)t * G + blockIdx.x) * kTile;
      if (tile0 + kTile > n4) break;
      f4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(in + tile0 + u * kBlock + threadIdx.x);
#pragma unroll
      for (int u = 0; u < 4; ++u) res[t * kTile + u * kBlock + threadIdx.x] = v[u];
    }
    __syncthreads();
    for (int t = 0; t < kTiles; ++t) {
      const size_t tile0 = lo + ((size_t)t * G + blockIdx.x) * kTile;
      if (tile0 + kTile > n4) break;
#pragma unroll
      for (int u = 0; u < 4; ++u)
        __builtin_nontemporal_store(res[t * kTile + u * kBlock + threadIdx.x], out + tile0 + u * kBlock + threadIdx.x);
    }
    __syncthreads();
  }
}

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

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 5;
  const size_t bytes = 4ull << 30, n4 = bytes / 16, R = bytes / 512;
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
  for (size_t r = 0; r < R; ++r) h[r] = gp_double_index{r, perm[r]};
  gp_double_index *idx;
  CK(hipMalloc(&idx, R * sizeof(gp_double_index)));
  CK(hipMemcpy(idx, h.data(), R * sizeof(gp_double_index), hipMemcpyHostToDevice));

  // correctness: every phased form == product on the same inputs (all floats)
  auto compare = [&](const char *what) {
    size_t bad = 0;
    std::vector<float> a(1 << 24), b(1 << 24);
    for (size_t off = 0; off < bytes / 4; off += a.size()) {
      CK(hipMemcpy(a.data(), y + off, a.size() * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(b.data(), y2 + off, b.size() * 4, hipMemcpyDeviceToHost));
      bad += std::memcmp(a.data(), b.data(), a.size() * 4) != 0;
    }
    std::printf("%s: phased vs product, %zu mismatching 64-MiB blocks\n", what, bad);
  };
  {
    CK(hipMemset(y, 0, bytes));
    CK(hipMemset(y2, 0, bytes));
    gp_gather_rows(y, x, idx, R, {0, 0}, 128, (size_t)-1, nullptr);
    launch_ph2<kAssignTo, 256, 288, 12>(y2, x, idx, R, 2);
    CK(hipDeviceSynchronize());
    compare("gather");
    gp_scatter_add_rows(y, x, idx, R, {0, 0}, 128, (size_t)-1, nullptr);
    launch_ph2<kAddFrom, 256, 288, 12>(y2, x, idx, R, 2);
    CK(hipDeviceSynchronize());
    compare("gather+add");
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
  vs.push_back(V{"copy ph160 k2", 2.0 * bytes, [=]() {
    const size_t G = num_cus(), chunk = G * 10240;
    for (size_t c = 0; c < (n4 + chunk - 1) / chunk; c += 2)
      copy_ph160<2><<<(unsigned)G, kBlock>>>(yv, xv, n4, c); }, {}});
  vs.push_back(V{"gather prod", gat_b, [=]() { gp_gather_rows(y, x, idx, R, {0, 0}, 128, (size_t)-1, nullptr); }, {}});
  vs.push_back(V{"gather ph2 B256 R288 S12 k2", gat_b, [=]() { launch_ph2<kAssignTo, 256, 288, 12>(y, x, idx, R, 2); }, {}});
  vs.push_back(V{"gather ph2 B256 R288 S12 k8", gat_b, [=]() { launch_ph2<kAssignTo, 256, 288, 12>(y, x, idx, R, 8); }, {}});
  vs.push_back(V{"gather ph2 B256 R288 S18 k2", gat_b, [=]() { launch_ph2<kAssignTo, 256, 288, 18>(y, x, idx, R, 2); }, {}});
  vs.push_back(V{"gather ph2 B256 R288 S36 k2", gat_b, [=]() { launch_ph2<kAssignTo, 256, 288, 36>(y, x, idx, R, 2); }, {}});
  vs.push_back(V{"gather ph2 B512 R288 S9 k2", gat_b, [=]() { launch_ph2<kAssignTo, 512, 288, 9>(y, x, idx, R, 2); }, {}});
  vs.push_back(V{"gather ph2 B512 R288 S18 k2", gat_b, [=]() { launch_ph2<kAssignTo, 512, 288, 18>(y, x, idx, R, 2); }, {}});
  vs.push_back(V{"gather ph2 B256 R128 S8 k4", gat_b, [=]() { launch_ph2<kAssignTo, 256, 128, 8>(y, x, idx, R, 4); }, {}});
  vs.push_back(V{"add prod", add_b, [=]() { gp_scatter_add_rows(y, x, idx, R, {0, 0}, 128, (size_t)-1, nullptr); }, {}});
  vs.push_back(V{"add ph2 B256 R288 S12 k2", add_b, [=]() { launch_ph2<kAddFrom, 256, 288, 12>(y, x, idx, R, 2); }, {}});
  vs.push_back(V{"add ph2 B256 R288 S12 k8", add_b, [=]() { launch_ph2<kAddFrom, 256, 288, 12>(y, x, idx, R, 8); }, {}});
  vs.push_back(V{"add ph2 B256 R288 S6 k2", add_b, [=]() { launch_ph2<kAddFrom, 256, 288, 6>(y, x, idx, R, 2); }, {}});
  vs.push_back(V{"add ph2 B512 R288 S9 k2", add_b, [=]() { launch_ph2<kAddFrom, 512, 288, 9>(y, x, idx, R, 2); }, {}});
  vs.push_back(V{"add ph2 B512 R288 S6 k2", add_b, [=]() { launch_ph2<kAddFrom, 512, 288, 6>(y, x, idx, R, 2); }, {}});
  vs.push_back(V{"init prod", gat_b, [=]() { gp_scatter_init_rows(y, x, idx, R, {0, 0}, 128, (size_t)-1, nullptr); }, {}});
  vs.push_back(V{"init ph2 B256 R288 S12 k2", gat_b, [=]() { launch_ph2<kInitFrom, 256, 288, 12>(y, x, idx, R, 2); }, {}});

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
  std::printf("%-30s %10s %10s %10s %8s\n", "variant", "med_ms", "min_ms", "GB/s", "frac8T");
  for (auto &v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const double med = v.ms[v.ms.size() / 2];
    const double gbs = v.bytes / (med * 1e-3) / 1e9;
    std::printf("%-30s %10.4f %10.4f %10.1f %8.4f\n", v.name.c_str(), med, v.ms[0], gbs, gbs / 8000.0);
  }
  return 0;
}
