// r3_tilemap_tune.hip — round-3 probe 8 (tuning harness, not product code; it
// #includes the product kernels): which 64-row tile each wave of the wave-map
// kernel (row_wave_kernel) takes, for the planned init / gather on a random
// index and on an identity index.
//   MAP 0  grid-stride, as production: wave w takes tiles w, w + waves, ...
//          (at any moment the chip writes one ~32-MiB window of the destination)
//   MAP 1  blocked: wave w takes a contiguous run of tiles (the chip writes
//          `waves` separate sequential streams spread over the whole buffer)
//   MAP 2  per XCD: blocks are dealt to the 8 XCDs round-robin, so XCD j
//          (blockIdx % 8) takes the j-th eighth of the tiles, grid-stride
//          inside it (each XCD's L2 sees one region)
// Same per-tile work as production: lane l resolves entry l of the tile, the
// next tile's entries load under this tile's rows, 8 rows in flight per
// 32-lane group, non-temporal accesses, one resident round of blocks.
// "prod kernel MAP0/2": the production row_wave_kernel with its MAP template
// argument (2 = the per-XCD map), launched directly on the sorted index.
// Every variant is bit-checked against the production planned call.
// Usage: r3_tilemap_tune [rounds]
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

// the k-th tile of wave `wave` (of `waves`) under MAP, or ~0 when done
template <int MAP>
__device__ __forceinline__ size_t tile_of(size_t wave, size_t waves, size_t k, size_t tiles) {
  if (MAP == 0) return wave + k * waves;
  if (MAP == 1) {
    const size_t per = (tiles + waves - 1) / waves;
    return k < per ? wave * per + k : ~size_t(0);
  }
  // MAP 2: wave = (block, wave-in-block); block b runs on XCD b % 8
  const size_t blk = wave / 4, wib = wave % 4, nblk = waves / 4;
  const size_t xcd = blk % 8, lb = blk / 8, per_xcd_blocks = nblk / 8;
  const size_t region = (tiles + 7) / 8;
  const size_t lw = lb * 4 + wib, lwaves = per_xcd_blocks * 4;
  const size_t i = lw + k * lwaves;
  return i < region ? xcd * region + i : ~size_t(0);
}

template <int OP, int MAP>
__global__ __launch_bounds__(kBlock) void map_kernel(float *__restrict__ y, const float *__restrict__ x,
                                                     const gp_double_index *__restrict__ index, size_t num_rows) {
  typedef __attribute__((address_space(1))) f4 GT;
  constexpr int LPR = 32, kG = 2, kRowsPerGroup = 32, kRPG = 8;
  const int wl = threadIdx.x & 63, lane = wl % LPR, gw = wl / LPR;
  const size_t wave = ((size_t)blockIdx.x * kBlock + threadIdx.x) / 64;
  const size_t waves = (size_t)gridDim.x * (kBlock / 64);
  const size_t tiles = (num_rows + 63) / 64;
  size_t k = 0, tile = tile_of<MAP>(wave, waves, k, tiles);
  if (tile >= tiles) return;
  uint64_t msrc = 0, mdst = 0;
  auto resolve = [&](size_t tl) {
    msrc = mdst = 0;
    const size_t e = tl * 64 + wl;
    if (tl >= tiles || e >= num_rows) return;
    const gp_double_index ix = index[e];
    uint64_t from, to;
    row_endpoints<OP>(ix, 0, 0, from, to);
    msrc = reinterpret_cast<uint64_t>(x + from * W);
    mdst = reinterpret_cast<uint64_t>(y + to * W);
  };
  resolve(tile);
  while (tile < tiles) {
    const size_t next = tile_of<MAP>(wave, waves, k + 1, tiles);
    uint64_t nsrc = 0, ndst = 0;
    {  // the next tile's entry, in flight meanwhile
      const size_t e = next * 64 + wl;
      if (next < tiles && e < num_rows) {
        const gp_double_index ix = index[e];
        uint64_t from, to;
        row_endpoints<OP>(ix, 0, 0, from, to);
        nsrc = reinterpret_cast<uint64_t>(x + from * W);
        ndst = reinterpret_cast<uint64_t>(y + to * W);
      }
    }
    const size_t rows_here = num_rows - tile * 64 < 64 ? num_rows - tile * 64 : 64;
    for (int i0 = 0; i0 < kRowsPerGroup; i0 += kRPG) {
      uint64_t sp[kRPG], dp[kRPG];
      bool live[kRPG];
      const uint64_t sp0 = shfl64(msrc, 0);  // the tile's first row: always there
#pragma unroll
      for (int q = 0; q < kRPG; ++q) {
        const int rt = gw + kG * (i0 + q);
        live[q] = (size_t)rt < rows_here;
        sp[q] = shfl64(msrc, rt);
        dp[q] = shfl64(mdst, rt);
        if (!live[q]) sp[q] = sp0;  // loads unconditional (a branch per load serialized them)
      }
      f4 xs[kRPG];
#pragma unroll
      for (int q = 0; q < kRPG; ++q) xs[q] = __builtin_nontemporal_load(reinterpret_cast<const GT *>(sp[q]) + lane);
      if (rows_here == 64) {  // wave-uniform: a whole tile, no per-row branches
#pragma unroll
        for (int q = 0; q < kRPG; ++q)
          __builtin_nontemporal_store(OP == kInitFrom ? f4(0.0f) + xs[q] : xs[q],
                                      reinterpret_cast<GT *>(dp[q]) + lane);
      } else {
#pragma unroll
        for (int q = 0; q < kRPG; ++q)
          if (live[q])
            __builtin_nontemporal_store(OP == kInitFrom ? f4(0.0f) + xs[q] : xs[q],
                                        reinterpret_cast<GT *>(dp[q]) + lane);
      }
    }
    msrc = nsrc;
    mdst = ndst;
    tile = next;
    ++k;
  }
}

__global__ void mismatch_kernel(const uint32_t *a, const uint32_t *b, size_t n, unsigned long long *cnt) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  unsigned long long c = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) c += a[i] != b[i];
  if (c) atomicAdd(cnt, c);
}

template <int OP, int MAP>
void launch_map(float *y, const float *x, const gp_double_index *ix, size_t n) {
  static std::atomic<int> occ{0};
  const int res = resident_blocks(reinterpret_cast<const void *>(&map_kernel<OP, MAP>), occ);
  // whole blocks per XCD for MAP 2: a multiple of 8 blocks
  size_t grid = (size_t)num_cus() * res;
  grid = grid / 8 * 8;
  hipLaunchKernelGGL((map_kernel<OP, MAP>), dim3((unsigned)grid), dim3(kBlock), 0, 0, y, x, ix, n);
}

// the production row_wave_kernel itself, MAP 0 or 2, one resident round of blocks
template <int OP, int MAP>
void launch_prod_map(float *y, const float *x, const gp_double_index *ix, size_t n) {
  auto *kern = &row_wave_kernel<f4, OP, 32, 8, kFlat, MAP>;
  static std::atomic<int> occ{0};
  size_t grid = (size_t)num_cus() * resident_blocks(reinterpret_cast<const void *>(kern), occ);
  grid = grid / 8 * 8;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(kBlock), 0, 0, y, x, ix, n, 0, 0, W, W / 4, ~size_t(0),
                     SegArg<kFlat>{});
}

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 5;
  std::mt19937_64 g(8);
  std::vector<uint64_t> perm(R);
  std::iota(perm.begin(), perm.end(), 0);
  std::shuffle(perm.begin(), perm.end(), g);
  // destination-sorted, as a plan's residual: gather {i, perm[i]}, init {perm[d], d}; identity
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
  gp_row_plan pg, pi;
  GK(gp_gather_plan_create(&pg, gat.data(), R, {0, 0}, W, ~size_t(0)));
  GK(gp_row_plan_create(&pi, ini.data(), R, {0, 0}, W, ~size_t(0)));
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
    for (size_t i = 0; i < N; i += 97) h[i] = -0.0f;
    CK(hipMemcpy(x, h.data(), N * 4, hipMemcpyHostToDevice));
  }
  struct V {
    std::string name;
    std::function<void()> f;
    int check;  // 1 gather, 2 init, 3 identity copy
  };
  std::vector<V> vs;
  vs.push_back({"gath prod (wave, plan)", [&] { gp_gather_rows_planned(y, x, pg, 0); }, 1});
  vs.push_back({"gath prod kernel MAP0", [&] { launch_prod_map<kAssignTo, 0>(y, x, igat, R); }, 1});
  vs.push_back({"gath prod kernel MAP2 (XCD)", [&] { launch_prod_map<kAssignTo, 2>(y, x, igat, R); }, 1});
  vs.push_back({"gath map0 grid-stride", [&] { launch_map<kAssignTo, 0>(y, x, igat, R); }, 1});
  vs.push_back({"gath map1 blocked", [&] { launch_map<kAssignTo, 1>(y, x, igat, R); }, 1});
  vs.push_back({"gath map2 per-XCD", [&] { launch_map<kAssignTo, 2>(y, x, igat, R); }, 1});
  vs.push_back({"init prod (wave, plan)", [&] { gp_scatter_init_rows_planned(y, x, pi, 0); }, 2});
  vs.push_back({"init prod kernel MAP0", [&] { launch_prod_map<kInitFrom, 0>(y, x, iini, R); }, 2});
  vs.push_back({"init prod kernel MAP2 (XCD)", [&] { launch_prod_map<kInitFrom, 2>(y, x, iini, R); }, 2});
  vs.push_back({"init map0 grid-stride", [&] { launch_map<kInitFrom, 0>(y, x, iini, R); }, 2});
  vs.push_back({"init map1 blocked", [&] { launch_map<kInitFrom, 1>(y, x, iini, R); }, 2});
  vs.push_back({"init map2 per-XCD", [&] { launch_map<kInitFrom, 2>(y, x, iini, R); }, 2});
  vs.push_back({"ident prod kernel MAP0", [&] { launch_prod_map<kAssignTo, 0>(y, x, iident, R); }, 3});
  vs.push_back({"ident prod kernel MAP2 (XCD)", [&] { launch_prod_map<kAssignTo, 2>(y, x, iident, R); }, 3});
  vs.push_back({"ident map0 grid-stride", [&] { launch_map<kAssignTo, 0>(y, x, iident, R); }, 3});
  vs.push_back({"ident map1 blocked", [&] { launch_map<kAssignTo, 1>(y, x, iident, R); }, 3});
  vs.push_back({"ident map2 per-XCD", [&] { launch_map<kAssignTo, 2>(y, x, iident, R); }, 3});

  for (int c = 1; c <= 3; ++c) {
    if (c == 1) GK(gp_gather_rows_planned(yr, x, pg, 0));
    if (c == 2) GK(gp_scatter_init_rows_planned(yr, x, pi, 0));
    if (c == 3) CK(hipMemcpy(yr, x, N * 4, hipMemcpyDeviceToDevice));
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
