// rowmap_tune.hip — A/B of the row-op kernel forms (tuning harness, not product
// code; it #includes the product kernels):
//   prod : row_op_kernel   — every lane of a row group loads the row's index entry
//   map  : row_map_kernel  — LDS-staged, double-buffered block index map
//   shfl : (here only)     — wave-level map: lane l loads row l's entry, the row
//                            groups get theirs by __shfl from that lane
// at several row widths, random-permutation DoubleIndex, plus sequential copy /
// add ceilings of the same byte counts.  Interleaved rounds in one process,
// median per variant.  All forms use the product's per-stream cache policy
// (ld_src / st_copy in gp_reduce.hip).  Usage: rowmap_tune [rounds]
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

// LDS-staged row-index map (the "map" form).  The block walks the DoubleIndex in tiles of
// kBlock rows: each thread loads ONE 16-B entry (a coalesced 4-KiB read per
// tile), resolves it to its (from, to) row pair and stores that in LDS; the row
// groups then read their rows' pairs from LDS (lanes of a group hit one
// address: a broadcast) instead of every lane re-loading the entry from global
// memory.  The map is double-buffered: the next tile's entries are loaded
// while this tile's rows move, so an index fetch never sits in front of the
// row loads it feeds.  Group g of the block takes tile rows g, g + kGroups, ...:
// consecutive groups take consecutive rows, so the x side of an identity-like
// index (Caffe's contiguous per-layer rows) stays contiguous across a wave.
template <typename T, int VEC, int OP, int LPR, int RPG>
__global__ __launch_bounds__(kBlock) void row_map_kernel(
    float *__restrict__ y, const float *__restrict__ x,
    const gp_double_index *__restrict__ index, size_t num_rows, uint64_t off0,
    uint64_t off1, size_t row_size, size_t vw, size_t limit) {
  constexpr int kGroups = kBlock / LPR;
  constexpr int kRowsPerGroup = kBlock / kGroups;  // == LPR
  constexpr int kRPG = RPG < kRowsPerGroup ? RPG : kRowsPerGroup;
  __shared__ uint64_t map_from[2][kBlock];
  __shared__ uint64_t map_to[2][kBlock];
  const int lane = threadIdx.x % LPR;
  const int grp = threadIdx.x / LPR;
  const size_t tstride = (size_t)gridDim.x * kBlock;
  size_t tile = (size_t)blockIdx.x * kBlock;
  if (tile >= num_rows) return;  // block-uniform: no barrier is skipped by part of a block
  T *yv = reinterpret_cast<T *>(y);
  const T *xv = reinterpret_cast<const T *>(x);

  {
    const size_t r = tile + threadIdx.x;
    if (r < num_rows) {
      uint64_t f, t;
      row_endpoints<OP>(index[r], off0, off1, f, t);
      map_from[0][threadIdx.x] = f;
      map_to[0][threadIdx.x] = t;
    }
  }
  __syncthreads();
  int buf = 0;
  for (; tile < num_rows; tile += tstride) {
    // prefetch the next tile's entry (in flight while this tile's rows move)
    const size_t nr = tile + tstride + threadIdx.x;
    const bool have_next = nr < num_rows;
    gp_double_index nix = {0, 0};
    if (have_next) nix = index[nr];
    const size_t rows_here = num_rows - tile < (size_t)kBlock ? num_rows - tile : (size_t)kBlock;

    for (int i0 = 0; i0 < kRowsPerGroup; i0 += kRPG) {
      uint64_t from[kRPG], to[kRPG];
      bool live[kRPG];
      bool all_whole = true;
#pragma unroll
      for (int k = 0; k < kRPG; ++k) {
        const size_t rt = (size_t)grp + (size_t)kGroups * (i0 + k);
        live[k] = rt < rows_here;
        from[k] = live[k] ? map_from[buf][rt] : 0;
        to[k] = live[k] ? map_to[buf][rt] : 0;
        const uint64_t guarded = (OP == kAssignTo) ? to[k] : from[k];
        all_whole = all_whole && (!live[k] || (guarded + 1) * row_size <= limit);
      }
      if (all_whole) {
        for (size_t j = lane; j < vw; j += LPR) {
          T xs[kRPG], ys[kRPG];
#pragma unroll
          for (int k = 0; k < kRPG; ++k)
            if (live[k]) xs[k] = ld_src<OP>(xv + from[k] * vw + j);
          if (OP == kAddFrom) {
#pragma unroll
            for (int k = 0; k < kRPG; ++k)
              if (live[k]) ys[k] = yv[to[k] * vw + j];
          }
#pragma unroll
          for (int k = 0; k < kRPG; ++k) {
            if (live[k]) {
              if (OP == kAddFrom)
                yv[to[k] * vw + j] = ys[k] + xs[k];
              else if (OP == kInitFrom)
                yv[to[k] * vw + j] = T(0.0f) + xs[k];  // == zerofy then +=, -0 -> +0 included
              else
                st_copy<OP>(yv + to[k] * vw + j, xs[k]);
            }
          }
        }
      } else {
        // Rows straddling num_vals_limit: element-wise guard, scalar accesses.
#pragma unroll 1
        for (int k = 0; k < kRPG; ++k) {
          if (!live[k]) continue;
          const uint64_t guarded = (OP == kAssignTo) ? to[k] : from[k];
          for (size_t e = lane; e < row_size; e += LPR) {
            if (guarded * row_size + e < limit) {
              const float xv1 = x[from[k] * row_size + e];
              if (OP == kAddFrom)
                y[to[k] * row_size + e] += xv1;
              else if (OP == kInitFrom)
                y[to[k] * row_size + e] = 0.0f + xv1;
              else
                y[to[k] * row_size + e] = xv1;
            } else if (OP == kInitFrom) {
              y[to[k] * row_size + e] = 0.0f;
            }
          }
        }
      }
    }
    if (have_next) {
      uint64_t f, t;
      row_endpoints<OP>(nix, off0, off1, f, t);
      map_from[buf ^ 1][threadIdx.x] = f;
      map_to[buf ^ 1][threadIdx.x] = t;
    }
    __syncthreads();
    buf ^= 1;
  }
}

// shfl64: the product's (gp_reduce.hip)

// Wave-level map (whole rows only: the harness never sets a limit).
template <int OP, int LPR, int RPG>
__global__ __launch_bounds__(kBlock) void row_shfl_kernel(float *__restrict__ y,
                                                          const float *__restrict__ x,
                                                          const gp_double_index *__restrict__ index,
                                                          size_t n, size_t vw) {
  constexpr int kG = 64 / LPR;
  constexpr int kRPG = RPG < LPR ? RPG : LPR;
  const int wl = threadIdx.x & 63, lane = wl % LPR, gw = wl / LPR;
  const size_t wave = ((size_t)blockIdx.x * kBlock + threadIdx.x) / 64;
  const size_t wstride = (size_t)gridDim.x * (kBlock / 64) * 64;
  f4 *yv = reinterpret_cast<f4 *>(y);
  const f4 *xv = reinterpret_cast<const f4 *>(x);
  size_t t = wave * 64;
  uint64_t mf = 0, mt = 0;
  if (t + wl < n) {
    const gp_double_index ix = index[t + wl];
    row_endpoints<OP>(ix, 0, 0, mf, mt);
  }
  for (; t < n; t += wstride) {
    const size_t nr = t + wstride + wl;
    gp_double_index nix = {0, 0};
    if (nr < n) nix = index[nr];
    const size_t rows_here = n - t < 64 ? n - t : 64;
    for (int i0 = 0; i0 < LPR; i0 += kRPG) {
      uint64_t from[kRPG], to[kRPG];
      bool live[kRPG];
#pragma unroll
      for (int k = 0; k < kRPG; ++k) {
        const int rt = gw + kG * (i0 + k);
        live[k] = (size_t)rt < rows_here;
        from[k] = shfl64(mf, rt);
        to[k] = shfl64(mt, rt);
      }
      for (size_t j = lane; j < vw; j += LPR) {
        f4 xs[kRPG], ys[kRPG];
#pragma unroll
        for (int k = 0; k < kRPG; ++k)
          if (live[k]) xs[k] = ld_src<OP>(xv + from[k] * vw + j);
        if (OP == kAddFrom) {
#pragma unroll
          for (int k = 0; k < kRPG; ++k)
            if (live[k]) ys[k] = yv[to[k] * vw + j];
        }
#pragma unroll
        for (int k = 0; k < kRPG; ++k)
          if (live[k]) st_copy<OP>(yv + to[k] * vw + j, OP == kAddFrom ? ys[k] + xs[k] : xs[k]);
      }
    }
    row_endpoints<OP>(nix, 0, 0, mf, mt);
  }
}

enum Form { kProd, kMap, kShfl };

template <int OP, int LPR, int RPG>
void launch(Form form, float *y, const float *x, const gp_double_index *idx, size_t n, size_t W,
            int per_cu) {
  const size_t cap = (size_t)num_cus() * per_cu;
  const size_t vw = W / 4;
  if (form == kProd) {
    constexpr int kGroups = kBlock / LPR;
    const size_t groups = (n + RPG - 1) / RPG;
    size_t grid = std::min((groups + kGroups - 1) / kGroups, cap);
    hipLaunchKernelGGL((row_op_kernel<f4, 4, OP, LPR, RPG>), dim3((unsigned)grid), dim3(kBlock), 0,
                       0, y, x, idx, n, 0, 0, W, vw, (size_t)-1);
  } else if (form == kMap) {
    size_t grid = std::min((n + kBlock - 1) / kBlock, cap);
    hipLaunchKernelGGL((row_map_kernel<f4, 4, OP, LPR, RPG>), dim3((unsigned)grid), dim3(kBlock), 0,
                       0, y, x, idx, n, 0, 0, W, vw, (size_t)-1);
  } else {
    size_t grid = std::min((n + kBlock - 1) / kBlock, cap);
    hipLaunchKernelGGL((row_shfl_kernel<OP, LPR, RPG>), dim3((unsigned)grid), dim3(kBlock), 0, 0,
                       y, x, idx, n, vw);
  }
}

__global__ void copy_k(f4 *__restrict__ out, const f4 *__restrict__ in, size_t n4) {
  const size_t stride = (size_t)gridDim.x * kBlock * 4;
  size_t i = (size_t)blockIdx.x * kBlock * 4 + threadIdx.x;
  for (; i + 3 * kBlock < n4; i += stride) {
    f4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(in + i + u * kBlock);
#pragma unroll
    for (int u = 0; u < 4; ++u) out[i + u * kBlock] = v[u];
  }
}

// the product's wave-map kernel at any op / lanes-per-row / rows in flight
template <int RPG, int LPR = 32, int OP = kAssignTo>
void launch_wave(float *y, const float *x, const gp_double_index *idx, size_t n, size_t W = 128) {
  size_t grid = std::min((n + kBlock - 1) / kBlock, grid_cap());
  hipLaunchKernelGGL((row_wave_kernel<f4, OP, LPR, RPG, kFlat>), dim3((unsigned)grid), dim3(kBlock),
                     0, 0, y, x, idx, n, 0, 0, W, W / 4, (size_t)-1, SegArg<kFlat>{});
}

gp_double_index *make_index(size_t R, uint64_t seed) {
  std::vector<uint64_t> perm(R);
  std::iota(perm.begin(), perm.end(), 0);
  std::mt19937_64 rng(seed);
  std::shuffle(perm.begin(), perm.end(), rng);
  std::vector<gp_double_index> h(R);
  for (size_t r = 0; r < R; ++r) h[r] = gp_double_index{r, perm[r]};
  gp_double_index *d;
  CK(hipMalloc(&d, R * sizeof(gp_double_index)));
  CK(hipMemcpy(d, h.data(), R * sizeof(gp_double_index), hipMemcpyHostToDevice));
  return d;
}

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 5;
  const size_t bytes = 4ull << 30;  // x and y: 4 GiB each (the 1M x 1024 table)
  float *x, *y;
  CK(hipMalloc(&x, bytes));
  CK(hipMalloc(&y, bytes));
  CK(hipMemset(x, 0, bytes));
  CK(hipMemset(y, 0, bytes));
  const size_t R128 = bytes / 512, R64 = bytes / 256, R1024 = bytes / 4096, R16 = bytes / 64;
  gp_double_index *i128 = make_index(R128, 5), *i64 = make_index(R64, 6),
                  *i1024 = make_index(R1024, 7), *i16 = make_index(R16, 8);

  struct V {
    std::string name;
    double bytes;
    std::function<void()> run;
    std::vector<float> ms;
  };
  std::vector<V> vs;
  auto add_b = [](size_t R, size_t W) { return 3.0 * R * W * 4 + 16.0 * R; };
  auto gat_b = [](size_t R, size_t W) { return 2.0 * R * W * 4 + 16.0 * R; };
#define ADD(NAME, B, ...) vs.push_back(V{NAME, B, [=]() { __VA_ARGS__; }, {}})
  if (std::getenv("ROWMAP_FOCUS")) {  // W = 128 gather / scatter-add: production vs shfl map
    gp_double_index *id128 = make_index(R128, 0);  // seed 0: shuffled too
    ADD("W128 gat prod L32R8", gat_b(R128, 128), (launch<kAssignTo, 32, 8>(kProd, y, x, i128, R128, 128, 8)));
    ADD("W128 gat shfl L32R8", gat_b(R128, 128), (launch<kAssignTo, 32, 8>(kShfl, y, x, i128, R128, 128, 8)));
    ADD("W128 gat C-ABI (wave R16)", gat_b(R128, 128), (gp_gather_rows(y, x, i128, R128, {0, 0}, 128, (size_t)-1, nullptr)));
    ADD("W128 gat wave R8", gat_b(R128, 128), (launch_wave<8>(y, x, i128, R128)));
    ADD("W128 gat shfl L32R4", gat_b(R128, 128), (launch<kAssignTo, 32, 4>(kShfl, y, x, i128, R128, 128, 8)));
    ADD("W128 gat shfl L32R16", gat_b(R128, 128), (launch<kAssignTo, 32, 16>(kShfl, y, x, i128, R128, 128, 8)));
    ADD("W128 gat shfl L32R8 x4", gat_b(R128, 128), (launch<kAssignTo, 32, 8>(kShfl, y, x, i128, R128, 128, 4)));
    ADD("W128 gat prod idx2", gat_b(R128, 128), (launch<kAssignTo, 32, 8>(kProd, y, x, id128, R128, 128, 8)));
    ADD("W128 gat shfl idx2", gat_b(R128, 128), (launch<kAssignTo, 32, 8>(kShfl, y, x, id128, R128, 128, 8)));
    ADD("W128 add prod L32R4", add_b(R128, 128), (launch<kAddFrom, 32, 4>(kProd, y, x, i128, R128, 128, 8)));
    ADD("W128 add shfl L32R4", add_b(R128, 128), (launch<kAddFrom, 32, 4>(kShfl, y, x, i128, R128, 128, 8)));
    ADD("W128 add shfl L32R8", add_b(R128, 128), (launch<kAddFrom, 32, 8>(kShfl, y, x, i128, R128, 128, 8)));
    ADD("W1024 gat prod L64R8", gat_b(R1024, 1024), (launch<kAssignTo, 64, 8>(kProd, y, x, i1024, R1024, 1024, 8)));
    ADD("W1024 gat shfl L64R8", gat_b(R1024, 1024), (launch<kAssignTo, 64, 8>(kShfl, y, x, i1024, R1024, 1024, 8)));
  } else if (std::getenv("ROWMAP_SCATTER")) {  // scatter-add / fused init: production vs wave map
    for (int rep = 0; rep < 2; ++rep) {
      ADD("W128 add C-ABI", add_b(R128, 128), (gp_scatter_add_rows(y, x, i128, R128, {0, 0}, 128, (size_t)-1, nullptr)));
      ADD("W128 add wave R4", add_b(R128, 128), (launch_wave<4, 32, kAddFrom>(y, x, i128, R128)));
      ADD("W128 add wave R8", add_b(R128, 128), (launch_wave<8, 32, kAddFrom>(y, x, i128, R128)));
      ADD("W128 init C-ABI", gat_b(R128, 128), (gp_scatter_init_rows(y, x, i128, R128, {0, 0}, 128, (size_t)-1, nullptr)));
      ADD("W128 init wave R8", gat_b(R128, 128), (launch_wave<8, 32, kInitFrom>(y, x, i128, R128)));
      ADD("W128 init wave R16", gat_b(R128, 128), (launch_wave<16, 32, kInitFrom>(y, x, i128, R128)));
      ADD("W64 add C-ABI", add_b(R64, 64), (gp_scatter_add_rows(y, x, i64, R64, {0, 0}, 64, (size_t)-1, nullptr)));
      ADD("W64 add wave R8", add_b(R64, 64), (launch_wave<8, 16, kAddFrom>(y, x, i64, R64, 64)));
      ADD("W64 init C-ABI", gat_b(R64, 64), (gp_scatter_init_rows(y, x, i64, R64, {0, 0}, 64, (size_t)-1, nullptr)));
      ADD("W64 init wave R16", gat_b(R64, 64), (launch_wave<16, 16, kInitFrom>(y, x, i64, R64, 64)));
    }
  } else if (std::getenv("ROWMAP_SHORT")) {  // gather of short rows: production vs maps
    ADD("W64 gat prod L16R8", gat_b(R64, 64), (launch<kAssignTo, 16, 8>(kProd, y, x, i64, R64, 64, 8)));
    ADD("W64 gat map  L16R8", gat_b(R64, 64), (launch<kAssignTo, 16, 8>(kMap, y, x, i64, R64, 64, 8)));
    ADD("W64 gat wave L16R8", gat_b(R64, 64), (launch_wave<8, 16>(y, x, i64, R64, 64)));
    ADD("W64 gat wave L16R16", gat_b(R64, 64), (launch_wave<16, 16>(y, x, i64, R64, 64)));
    ADD("W16 gat prod L4R8", gat_b(R16, 16), (launch<kAssignTo, 4, 8>(kProd, y, x, i16, R16, 16, 8)));
    ADD("W16 gat map  L4R8", gat_b(R16, 16), (launch<kAssignTo, 4, 8>(kMap, y, x, i16, R16, 16, 8)));
    ADD("W16 gat wave L4R4", gat_b(R16, 16), (launch_wave<4, 4>(y, x, i16, R16, 16)));
    ADD("W128 gat wave L32R8", gat_b(R128, 128), (launch_wave<8, 32>(y, x, i128, R128, 128)));
    ADD("W128 gat prod L32R8", gat_b(R128, 128), (launch<kAssignTo, 32, 8>(kProd, y, x, i128, R128, 128, 8)));
  } else {
    ADD("W128 add prod L32R4", add_b(R128, 128), (launch<kAddFrom, 32, 4>(kProd, y, x, i128, R128, 128, 8)));
    ADD("W128 add map  L32R4", add_b(R128, 128), (launch<kAddFrom, 32, 4>(kMap, y, x, i128, R128, 128, 8)));
    ADD("W128 add map  L32R8", add_b(R128, 128), (launch<kAddFrom, 32, 8>(kMap, y, x, i128, R128, 128, 8)));
    ADD("W128 add map  L32R4 pc4", add_b(R128, 128), (launch<kAddFrom, 32, 4>(kMap, y, x, i128, R128, 128, 4)));
    ADD("W128 add shfl L32R4", add_b(R128, 128), (launch<kAddFrom, 32, 4>(kShfl, y, x, i128, R128, 128, 8)));
    ADD("W128 gat prod L32R8", gat_b(R128, 128), (launch<kAssignTo, 32, 8>(kProd, y, x, i128, R128, 128, 8)));
    ADD("W128 gat map  L32R8", gat_b(R128, 128), (launch<kAssignTo, 32, 8>(kMap, y, x, i128, R128, 128, 8)));
    ADD("W128 gat map  L32R4", gat_b(R128, 128), (launch<kAssignTo, 32, 4>(kMap, y, x, i128, R128, 128, 8)));
    ADD("W128 gat shfl L32R8", gat_b(R128, 128), (launch<kAssignTo, 32, 8>(kShfl, y, x, i128, R128, 128, 8)));
    ADD("W128 init prod L32R8", gat_b(R128, 128), (launch<kInitFrom, 32, 8>(kProd, y, x, i128, R128, 128, 8)));
    ADD("W128 init map  L32R8", gat_b(R128, 128), (launch<kInitFrom, 32, 8>(kMap, y, x, i128, R128, 128, 8)));
    ADD("W64 add prod L16R4", add_b(R64, 64), (launch<kAddFrom, 16, 4>(kProd, y, x, i64, R64, 64, 8)));
    ADD("W64 add map  L16R4", add_b(R64, 64), (launch<kAddFrom, 16, 4>(kMap, y, x, i64, R64, 64, 8)));
    ADD("W64 add shfl L16R4", add_b(R64, 64), (launch<kAddFrom, 16, 4>(kShfl, y, x, i64, R64, 64, 8)));
    ADD("W64 gat prod L16R8", gat_b(R64, 64), (launch<kAssignTo, 16, 8>(kProd, y, x, i64, R64, 64, 8)));
    ADD("W64 gat map  L16R8", gat_b(R64, 64), (launch<kAssignTo, 16, 8>(kMap, y, x, i64, R64, 64, 8)));
    ADD("W16 add prod L4R4", add_b(R16, 16), (launch<kAddFrom, 4, 4>(kProd, y, x, i16, R16, 16, 8)));
    ADD("W16 add map  L4R4", add_b(R16, 16), (launch<kAddFrom, 4, 4>(kMap, y, x, i16, R16, 16, 8)));
    ADD("W16 add shfl L4R4", add_b(R16, 16), (launch<kAddFrom, 4, 4>(kShfl, y, x, i16, R16, 16, 8)));
    ADD("W16 gat prod L4R8", gat_b(R16, 16), (launch<kAssignTo, 4, 8>(kProd, y, x, i16, R16, 16, 8)));
    ADD("W16 gat map  L4R8", gat_b(R16, 16), (launch<kAssignTo, 4, 8>(kMap, y, x, i16, R16, 16, 8)));
    ADD("W1024 add prod L64R4", add_b(R1024, 1024), (launch<kAddFrom, 64, 4>(kProd, y, x, i1024, R1024, 1024, 8)));
    ADD("W1024 add map  L64R4", add_b(R1024, 1024), (launch<kAddFrom, 64, 4>(kMap, y, x, i1024, R1024, 1024, 8)));
    ADD("W1024 gat prod L64R8", gat_b(R1024, 1024), (launch<kAssignTo, 64, 8>(kProd, y, x, i1024, R1024, 1024, 8)));
    ADD("W1024 gat map  L64R8", gat_b(R1024, 1024), (launch<kAssignTo, 64, 8>(kMap, y, x, i1024, R1024, 1024, 8)));
  // ceilings: sequential streams of the same bytes
  }
  ADD("ceil copy 1R1W (kernel)", 2.0 * bytes,
      (copy_k<<<num_cus() * 8, kBlock>>>(reinterpret_cast<f4 *>(y), reinterpret_cast<const f4 *>(x), bytes / 16)));
  ADD("ceil add 2R1W (gp_add)", 3.0 * bytes, (gp_add(bytes / 4, y, x, y, nullptr)));

  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (auto &v : vs) v.run();
  CK(hipDeviceSynchronize());
  for (int r = 0; r < rounds; ++r) {
    for (auto &v : vs) {
      CK(hipEventRecord(a));
      v.run();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      v.ms.push_back(ms);
    }
    std::fprintf(stderr, "round %d done\n", r);
  }
  std::printf("%-28s %10s %10s %10s %8s\n", "variant", "med_ms", "min_ms", "GB/s", "frac8T");
  for (auto &v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const double med = v.ms[v.ms.size() / 2];
    const double gbs = v.bytes / (med * 1e-3) / 1e9;
    std::printf("%-28s %10.4f %10.4f %10.1f %8.4f\n", v.name.c_str(), med, v.ms[0], gbs, gbs / 8000.0);
  }
  return 0;
}
