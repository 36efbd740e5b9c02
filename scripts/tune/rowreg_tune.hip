// rowreg_tune.hip — probe: a register-phased scatter-add / fused init of
// 128-float rows (tuning harness, not product code; it #includes the product
// kernels for the A/B).
//
// The 8-way sum gains 10-25 % when the chip reads in one phase and writes in the
// next.  The earlier row-op phase probes (rowphase*_tune.hip) parked
// rows in LDS at one block per CU and could not keep enough random rows in
// flight.  Here each wave parks its rows in REGISTERS: a 32-lane group owns one
// 512-B row per f4 lane, K rows per group, 2 groups per wave.  The wave loads
// its 2K index entries in one coalesced read (one per lane, resolved by shfl),
// issues every x and y load of its rows, adds, then (optionally after a block
// barrier) stores.  One launch covers one chunk (grid x waves x 2K rows) so the
// launch boundary keeps the whole chip in phase, as the phased bucket sum does.
// Usage: rowreg_tune [rounds]
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

template <int OP, int BLK, int K, bool SYNC>
__global__ __launch_bounds__(BLK) void row_regphase_kernel(float *__restrict__ y,
                                                           const float *__restrict__ x,
                                                           const gp_double_index *__restrict__ idx,
                                                           size_t n) {
  static_assert(2 * K <= 64, "one index entry per lane");
  const int wl = threadIdx.x & 63, lane = wl & 31, gw = wl >> 5;
  const size_t wave = ((size_t)blockIdx.x * BLK + threadIdx.x) >> 6;
  const size_t base = wave * (2 * K);
  uint64_t mf = 0, mt = 0;
  if (wl < 2 * K && base + wl < n) {
    const gp_double_index ix = idx[base + wl];
    mf = ix.id0;
    mt = ix.id1;
  }
  f4 *yv = reinterpret_cast<f4 *>(y);
  const f4 *xv = reinterpret_cast<const f4 *>(x);
  f4 xs[K], s[K];
  uint64_t to[K];
  bool live[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int rt = gw * K + k;
    live[k] = base + rt < n;
    const uint64_t from = shfl64(mf, rt);
    to[k] = shfl64(mt, rt);
    if (live[k]) xs[k] = __builtin_nontemporal_load(xv + from * 32 + lane);
  }
  if (OP == kAddFrom) {
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (live[k]) s[k] = yv[to[k] * 32 + lane];
  }
#pragma unroll
  for (int k = 0; k < K; ++k) s[k] = (OP == kAddFrom ? s[k] : f4(0.0f)) + xs[k];
  if (SYNC) __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k)
    if (live[k]) yv[to[k] * 32 + lane] = s[k];
}

template <int OP, int BLK, int K, bool SYNC>
void launch_reg(float *y, const float *x, const gp_double_index *idx, size_t n, int per_cu) {
  const size_t grid = (size_t)num_cus() * per_cu;
  const size_t chunk = grid * (BLK / 64) * 2 * K;
  for (size_t c = 0; c < n; c += chunk) {
    const size_t m = std::min(chunk, n - c);
    const size_t g = std::min(grid, (m + (BLK / 64) * 2 * K - 1) / ((BLK / 64) * 2 * K));
    hipLaunchKernelGGL((row_regphase_kernel<OP, BLK, K, SYNC>), dim3((unsigned)g), dim3(BLK), 0, 0,
                       y, x, idx + c, m);
  }
}

__global__ void fill_k(float *p, size_t n, uint32_t seed) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    p[i] = (float)(h & 0xffffff) / 16777216.0f - 0.5f;
  }
}

gp_double_index *make_index(size_t R, uint64_t seed, bool identity) {
  std::vector<uint64_t> perm(R);
  std::iota(perm.begin(), perm.end(), 0);
  if (!identity) {
    std::mt19937_64 rng(seed);
    std::shuffle(perm.begin(), perm.end(), rng);
  }
  std::vector<gp_double_index> h(R);
  for (size_t r = 0; r < R; ++r) h[r] = gp_double_index{r, perm[r]};
  gp_double_index *d;
  CK(hipMalloc(&d, R * sizeof(gp_double_index)));
  CK(hipMemcpy(d, h.data(), R * sizeof(gp_double_index), hipMemcpyHostToDevice));
  return d;
}

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 5;
  const size_t bytes = 4ull << 30;  // x and y: 4 GiB each (the 1M x 1024 table as RowData rows)
  const size_t R = bytes / 512;
  float *x, *y, *y0, *yref;
  CK(hipMalloc(&x, bytes));
  CK(hipMalloc(&y, bytes));
  CK(hipMalloc(&y0, bytes));
  CK(hipMalloc(&yref, bytes));
  hipLaunchKernelGGL(fill_k, dim3(4096), dim3(256), 0, 0, x, bytes / 4, 11u);
  hipLaunchKernelGGL(fill_k, dim3(4096), dim3(256), 0, 0, y0, bytes / 4, 12u);
  gp_double_index *ir = make_index(R, 5, false), *ii = make_index(R, 0, true);

  struct V {
    std::string name;
    double bytes;
    std::function<void(float *, const gp_double_index *)> run;
    int op;
    std::vector<float> ms;
  };
  std::vector<V> vs;
  const double add_b = 3.0 * bytes + 16.0 * R, init_b = 2.0 * bytes + 16.0 * R;
#define ADD(NAME, B, OPV, ...) \
  vs.push_back(V{NAME, B, [=](float *yy, const gp_double_index *ix) { __VA_ARGS__; }, OPV, {}})
  ADD("add C-ABI", add_b, kAddFrom, (gp_scatter_add_rows(yy, x, ix, R, {0, 0}, 128, (size_t)-1, nullptr)));
  ADD("add reg B512 K16 c1", add_b, kAddFrom, (launch_reg<kAddFrom, 512, 16, false>(yy, x, ix, R, 1)));
  ADD("add reg B512 K16 c1 sync", add_b, kAddFrom, (launch_reg<kAddFrom, 512, 16, true>(yy, x, ix, R, 1)));
  ADD("add reg B512 K16 c2", add_b, kAddFrom, (launch_reg<kAddFrom, 512, 16, false>(yy, x, ix, R, 2)));
  ADD("add reg B512 K16 c2 sync", add_b, kAddFrom, (launch_reg<kAddFrom, 512, 16, true>(yy, x, ix, R, 2)));
  ADD("add reg B256 K16 c4", add_b, kAddFrom, (launch_reg<kAddFrom, 256, 16, false>(yy, x, ix, R, 4)));
  ADD("add reg B1024 K8 c1 sync", add_b, kAddFrom, (launch_reg<kAddFrom, 1024, 8, true>(yy, x, ix, R, 1)));
  ADD("add reg B256 K8 c8", add_b, kAddFrom, (launch_reg<kAddFrom, 256, 8, false>(yy, x, ix, R, 8)));
  ADD("add reg B512 K24 c1 sync", add_b, kAddFrom, (launch_reg<kAddFrom, 512, 24, true>(yy, x, ix, R, 1)));
  ADD("add reg B256 K32 c2", add_b, kAddFrom, (launch_reg<kAddFrom, 256, 32, false>(yy, x, ix, R, 2)));
  ADD("init C-ABI", init_b, kInitFrom, (gp_scatter_init_rows(yy, x, ix, R, {0, 0}, 128, (size_t)-1, nullptr)));
  ADD("init reg B512 K16 c2", init_b, kInitFrom, (launch_reg<kInitFrom, 512, 16, false>(yy, x, ix, R, 2)));
  ADD("init reg B512 K16 c1 sync", init_b, kInitFrom, (launch_reg<kInitFrom, 512, 16, true>(yy, x, ix, R, 1)));
  ADD("init reg B256 K32 c2", init_b, kInitFrom, (launch_reg<kInitFrom, 256, 32, false>(yy, x, ix, R, 2)));

  // parity: every variant vs the product on the same y0, random and identity index
  std::vector<uint32_t> a(bytes / 4), b(bytes / 4);
  for (const gp_double_index *ix : {ir, ii}) {
    for (int op : {(int)kAddFrom, (int)kInitFrom}) {
      CK(hipMemcpy(yref, y0, bytes, hipMemcpyDeviceToDevice));
      for (auto &v : vs)
        if (v.op == op && v.name.find("C-ABI") != std::string::npos) v.run(yref, ix);
      CK(hipMemcpy(a.data(), yref, bytes, hipMemcpyDeviceToHost));
      for (auto &v : vs) {
        if (v.op != op || v.name.find("C-ABI") != std::string::npos) continue;
        CK(hipMemcpy(y, y0, bytes, hipMemcpyDeviceToDevice));
        v.run(y, ix);
        CK(hipMemcpy(b.data(), y, bytes, hipMemcpyDeviceToHost));
        if (std::memcmp(a.data(), b.data(), bytes) != 0) {
          std::printf("MISMATCH %s (%s index)\n", v.name.c_str(), ix == ir ? "random" : "identity");
          return 3;
        }
      }
    }
  }
  std::printf("parity: every variant bit-identical to the product (random + identity index)\n");

  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<V> all;
  for (const char *tag : {"random", "ident"}) {
    for (auto v : vs) {
      v.name = std::string(tag) + " " + v.name;
      all.push_back(v);
    }
  }
  for (auto &v : all) v.run(y, v.name[0] == 'r' ? ir : ii);
  CK(hipDeviceSynchronize());
  for (int r = 0; r < rounds; ++r) {
    for (auto &v : all) {
      const gp_double_index *ix = v.name[0] == 'r' ? ir : ii;
      CK(hipEventRecord(e0));
      v.run(y, ix);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.ms.push_back(ms);
    }
    std::fprintf(stderr, "round %d done\n", r);
  }
  std::printf("%-34s %10s %10s %10s %8s\n", "variant", "med_ms", "min_ms", "GB/s", "frac8T");
  for (auto &v : all) {
    std::sort(v.ms.begin(), v.ms.end());
    const double med = v.ms[v.ms.size() / 2];
    const double gbs = v.bytes / (med * 1e-3) / 1e9;
    std::printf("%-34s %10.4f %10.4f %10.1f %8.4f\n", v.name.c_str(), med, v.ms[0], gbs, gbs / 8000.0);
  }
  return 0;
}
