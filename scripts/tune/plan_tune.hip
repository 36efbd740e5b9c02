// plan_tune.hip — A/B of the client accumulate forms behind gp_row_plan
// (tuning harness, not product code; it #includes the product kernels).
// 8 M rows of 128 floats (the 1M x 1024 table through the API), 4 GiB op
// buffer x, 4 GiB oplog y:
//   add/init  rand  : random-permutation DoubleIndex (row_op_kernel, production
//                     gp_scatter_add_rows / gp_scatter_init_rows)
//   add/init  rand-pf : row_op_kernel with the next iteration's index entries
//                     loaded before this iteration's rows move (here only)
//   add/init  sorted  : the same permutation sorted by id1 (what a plan's
//                     residual holds), row_op_kernel / row_wave_kernel / pf
//   add  ident-dense : identity index as one dense run (launch_bucket_sum_nb<1>;
//                     the plan's dense form while it had one.  An init twin of
//                     it, out = 0.0f + x through the sum kernels with the
//                     master read dropped, ran at 71 %: profiles/r02/plan_tune*.txt)
//   copy      : hipMemcpy D2D of 4 GiB (1 read + 1 write ceiling)
// Interleaved rounds in one process, median per variant.  Usage: plan_tune [rounds]
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

// row_op_kernel (whole rows only, no limit) with the next iteration's index
// entries in flight while this iteration's rows move.
template <int OP, int LPR, int RPG>
__global__ __launch_bounds__(kBlock) void row_op_pf_kernel(float *__restrict__ y,
                                                           const float *__restrict__ x,
                                                           const gp_double_index *__restrict__ index,
                                                           size_t num_rows, size_t vw) {
  constexpr int kGroups = kBlock / LPR;
  const int lane = threadIdx.x % LPR;
  const size_t group = (size_t)blockIdx.x * kGroups + threadIdx.x / LPR;
  const size_t gstride = (size_t)gridDim.x * kGroups * RPG;
  f4 *yv = reinterpret_cast<f4 *>(y);
  const f4 *xv = reinterpret_cast<const f4 *>(x);
  gp_double_index cur[RPG];
  size_t r0 = group * RPG;
#pragma unroll
  for (int k = 0; k < RPG; ++k) cur[k] = r0 + k < num_rows ? index[r0 + k] : gp_double_index{0, 0};
  for (; r0 < num_rows; r0 += gstride) {
    gp_double_index nxt[RPG];
    const size_t r1 = r0 + gstride;
#pragma unroll
    for (int k = 0; k < RPG; ++k) nxt[k] = r1 + k < num_rows ? index[r1 + k] : gp_double_index{0, 0};
    bool live[RPG];
#pragma unroll
    for (int k = 0; k < RPG; ++k) live[k] = r0 + k < num_rows;
    for (size_t j = lane; j < vw; j += LPR) {
      f4 xs[RPG], ys[RPG];
#pragma unroll
      for (int k = 0; k < RPG; ++k)
        if (live[k]) xs[k] = __builtin_nontemporal_load(xv + cur[k].id0 * vw + j);
      if (OP == kAddFrom) {
#pragma unroll
        for (int k = 0; k < RPG; ++k)
          if (live[k]) ys[k] = yv[cur[k].id1 * vw + j];
      }
#pragma unroll
      for (int k = 0; k < RPG; ++k)
        if (live[k]) yv[cur[k].id1 * vw + j] = OP == kAddFrom ? ys[k] + xs[k] : f4(0.0f) + xs[k];
    }
#pragma unroll
    for (int k = 0; k < RPG; ++k) cur[k] = nxt[k];
  }
}

// row_op_kernel shape (whole rows, no limit) with the oplog side's cache
// policy as parameters: YL / YS = non-temporal y loads / stores.
template <int OP, int LPR, int RPG, bool YL, bool YS>
__global__ __launch_bounds__(kBlock) void row_var_kernel(float *__restrict__ y,
                                                         const float *__restrict__ x,
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
      live[k] = r0 + k < num_rows;
      from[k] = to[k] = 0;
      if (live[k]) {
        const gp_double_index ix = index[r0 + k];
        from[k] = ix.id0;
        to[k] = ix.id1;
      }
    }
    for (size_t j = lane; j < vw; j += LPR) {
      f4 xs[RPG], ys[RPG];
#pragma unroll
      for (int k = 0; k < RPG; ++k)
        if (live[k]) xs[k] = __builtin_nontemporal_load(xv + from[k] * vw + j);
      if (OP == kAddFrom) {
#pragma unroll
        for (int k = 0; k < RPG; ++k)
          if (live[k]) ys[k] = YL ? __builtin_nontemporal_load(yv + to[k] * vw + j) : yv[to[k] * vw + j];
      }
#pragma unroll
      for (int k = 0; k < RPG; ++k)
        if (live[k]) {
          const f4 v = OP == kAddFrom ? ys[k] + xs[k] : f4(0.0f) + xs[k];
          if (YS)
            __builtin_nontemporal_store(v, yv + to[k] * vw + j);
          else
            yv[to[k] * vw + j] = v;
        }
    }
  }
}

// row_wave_kernel shape (flat, whole rows, LPR 32) with the oplog side's
// cache policy as parameters.
template <int OP, int RPG, bool YL, bool YS>
__global__ __launch_bounds__(kBlock) void wave_var_kernel(float *__restrict__ y,
                                                          const float *__restrict__ x,
                                                          const gp_double_index *__restrict__ index,
                                                          size_t num_rows, size_t vw) {
  typedef __attribute__((address_space(1))) f4 GT;
  constexpr int LPR = 32, kG = 2, kRowsPerGroup = 32;
  const int wl = threadIdx.x & 63, lane = wl % LPR, gw = wl / LPR;
  const size_t wave = ((size_t)blockIdx.x * kBlock + threadIdx.x) / 64;
  const size_t wstride = (size_t)gridDim.x * (kBlock / 64) * 64;
  size_t t = wave * 64;
  if (t >= num_rows) return;
  uint64_t msrc = 0, mdst = 0;
  auto resolve = [&](const gp_double_index &ix, bool live) {
    msrc = live ? reinterpret_cast<uint64_t>(x + ix.id0 * 128) : 0;
    mdst = live ? reinterpret_cast<uint64_t>(y + ix.id1 * 128) : 0;
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
      uint64_t sp[RPG], dp[RPG];
      bool live[RPG];
#pragma unroll
      for (int k = 0; k < RPG; ++k) {
        const int rt = gw + kG * (i0 + k);
        live[k] = (size_t)rt < rows_here;
        sp[k] = shfl64(msrc, rt);
        dp[k] = shfl64(mdst, rt);
      }
      for (size_t j = lane; j < vw; j += LPR) {
        f4 xs[RPG], ys[RPG];
#pragma unroll
        for (int k = 0; k < RPG; ++k)
          if (live[k]) xs[k] = __builtin_nontemporal_load(reinterpret_cast<const GT *>(sp[k]) + j);
        if (OP == kAddFrom) {
#pragma unroll
          for (int k = 0; k < RPG; ++k)
            if (live[k])
              ys[k] = YL ? __builtin_nontemporal_load(reinterpret_cast<const GT *>(dp[k]) + j)
                         : reinterpret_cast<const GT *>(dp[k])[j];
        }
#pragma unroll
        for (int k = 0; k < RPG; ++k) {
          if (!live[k]) continue;
          GT *d = reinterpret_cast<GT *>(dp[k]) + j;
          const f4 v = OP == kAddFrom ? ys[k] + xs[k] : f4(0.0f) + xs[k];
          if (YS)
            __builtin_nontemporal_store(v, d);
          else
            *d = v;
        }
      }
    }
    resolve(nix, nlive);
  }
}

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 5;
  const size_t R = 1u << 23, W = 128, n = R * W;
  float *x, *y;
  gp_double_index *rnd, *srt, *idn;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&y, n * 4));
  CK(hipMalloc(&rnd, R * 16));
  CK(hipMalloc(&srt, R * 16));
  CK(hipMalloc(&idn, R * 16));
  {
    std::vector<float> h(n);
    std::mt19937 g(3);
    std::uniform_real_distribution<float> d(-0.5f, 0.5f);
    for (auto &v : h) v = d(g);
    CK(hipMemcpy(x, h.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(y, h.data(), n * 4, hipMemcpyHostToDevice));
    std::vector<uint64_t> perm(R);
    std::iota(perm.begin(), perm.end(), 0);
    std::shuffle(perm.begin(), perm.end(), g);
    std::vector<gp_double_index> a(R), b(R), c(R);
    for (size_t r = 0; r < R; ++r) {
      a[r] = {r, perm[r]};
      b[perm[r]] = {r, perm[r]};  // sorted by id1
      c[r] = {r, r};
    }
    CK(hipMemcpy(rnd, a.data(), R * 16, hipMemcpyHostToDevice));
    CK(hipMemcpy(srt, b.data(), R * 16, hipMemcpyHostToDevice));
    CK(hipMemcpy(idn, c.data(), R * 16, hipMemcpyHostToDevice));
  }
  const size_t cap = grid_cap();
  auto rowop = [&](int op, const gp_double_index *ix) {
    return [=] {
      if (op == kAddFrom)
        launch_row_op<kAddFrom>(y, x, ix, R, {0, 0}, W, ~size_t(0), 0);
      else if (op == kAssignTo)
        launch_row_op<kAssignTo>(x, y, ix, R, {0, 0}, W, ~size_t(0), 0);
      else
        launch_row_op<kInitFrom>(y, x, ix, R, {0, 0}, W, ~size_t(0), 0);
    };
  };
  auto prod_sorted = [&](int op, const gp_double_index *ix) {
    return [=] {
      if (op == kAddFrom)
        launch_row_op<kAddFrom>(y, x, ix, R, {0, 0}, W, ~size_t(0), 0, true);
      else
        launch_row_op<kInitFrom>(y, x, ix, R, {0, 0}, W, ~size_t(0), 0, true);
    };
  };
  auto wave = [&](int op, const gp_double_index *ix) {
    return [=] {
      size_t grid = std::min((R + kBlock - 1) / kBlock, cap);
      const SegArg<kFlat> flat{};
      if (op == kAddFrom)
        hipLaunchKernelGGL((row_wave_kernel<f4, kAddFrom, 32, 8, kFlat>), dim3(grid), dim3(kBlock), 0,
                           0, y, x, ix, R, 0, 0, W, W / 4, ~size_t(0), flat);
      else
        hipLaunchKernelGGL((row_wave_kernel<f4, kInitFrom, 32, 8, kFlat>), dim3(grid), dim3(kBlock),
                           0, 0, y, x, ix, R, 0, 0, W, W / 4, ~size_t(0), flat);
    };
  };
  auto pf = [&](int op, const gp_double_index *ix, int rpg) {
    return [=] {
      const size_t groups = (R + rpg - 1) / rpg;
      size_t grid = std::min((groups + 7) / 8, cap);
      if (op == kAddFrom && rpg == 4)
        hipLaunchKernelGGL((row_op_pf_kernel<kAddFrom, 32, 4>), dim3(grid), dim3(kBlock), 0, 0, y, x,
                           ix, R, W / 4);
      else if (op == kAddFrom)
        hipLaunchKernelGGL((row_op_pf_kernel<kAddFrom, 32, 2>), dim3(grid), dim3(kBlock), 0, 0, y, x,
                           ix, R, W / 4);
      else
        hipLaunchKernelGGL((row_op_pf_kernel<kInitFrom, 32, 8>), dim3(grid), dim3(kBlock), 0, 0, y,
                           x, ix, R, W / 4);
    };
  };
  auto var = [&](int op, const gp_double_index *ix, int rpg, bool yl, bool ys, int per_cu) {
    return [=] {
      const size_t groups = (R + rpg - 1) / rpg;
      size_t grid = std::min((groups + 7) / 8, (size_t)num_cus() * per_cu);
#define VAR(OPV, RPGV, YLV, YSV)                                                                \
  if (op == OPV && rpg == RPGV && yl == YLV && ys == YSV)                                       \
    hipLaunchKernelGGL((row_var_kernel<OPV, 32, RPGV, YLV, YSV>), dim3(grid), dim3(kBlock), 0, 0, y, \
                       x, ix, R, W / 4);
      VAR(kAddFrom, 4, false, false)
      VAR(kAddFrom, 4, true, true)
      VAR(kAddFrom, 4, false, true)
      VAR(kAddFrom, 4, true, false)
      VAR(kAddFrom, 8, false, false)
      VAR(kAddFrom, 8, true, true)
      VAR(kAddFrom, 2, true, true)
      VAR(kInitFrom, 8, false, false)
      VAR(kInitFrom, 8, false, true)
      VAR(kInitFrom, 4, false, true)
#undef VAR
    };
  };
  auto wvar = [&](int op, const gp_double_index *ix, int rpg, bool yl, bool ys, int per_cu) {
    return [=] {
      size_t grid = std::min((R + kBlock - 1) / kBlock, (size_t)num_cus() * per_cu);
#define WVAR(OPV, RPGV, YLV, YSV)                                                               \
  if (op == OPV && rpg == RPGV && yl == YLV && ys == YSV)                                       \
    hipLaunchKernelGGL((wave_var_kernel<OPV, RPGV, YLV, YSV>), dim3(grid), dim3(kBlock), 0, 0, y, x, \
                       ix, R, W / 4);
      WVAR(kAddFrom, 8, true, true)
      WVAR(kAddFrom, 8, false, true)
      WVAR(kAddFrom, 4, true, true)
      WVAR(kAddFrom, 8, false, false)
      WVAR(kInitFrom, 8, false, true)
      WVAR(kInitFrom, 16, false, true)
      WVAR(kInitFrom, 4, false, true)
#undef WVAR
    };
  };
  auto gath = [&](const gp_double_index *ix, int per_cu) {
    return [=] {
      size_t grid = std::min((R + kBlock - 1) / kBlock, (size_t)num_cus() * per_cu);
      const SegArg<kFlat> flat{};
      hipLaunchKernelGGL((row_wave_kernel<f4, kAssignTo, 32, 8, kFlat>), dim3(grid), dim3(kBlock), 0, 0,
                         x, y, ix, R, 0, 0, W, W / 4, ~size_t(0), flat);
    };
  };
  auto dense_add = [&] {
    BucketPtrs b = {};
    b.p[0] = x;
    launch_bucket_sum_nb<1>(y, y, b, n, 0);
  };
  auto copy = [&] { CK(hipMemcpyAsync(y, x, n * 4, hipMemcpyDeviceToDevice, 0)); };
  const double add_b = 3.0 * n * 4 + 16.0 * R, init_b = 2.0 * n * 4 + 16.0 * R;
  struct V {
    std::string name;
    std::function<void()> f;
    double bytes;
  };
  const double gat_b = 2.0 * n * 4 + 16.0 * R;
  std::vector<V> vs = {
      {"add  rand   row_op (prod)", rowop(kAddFrom, rnd), add_b},
      {"add  ident  dense", dense_add, 3.0 * n * 4},
      {"add  ident  prod sorted (wave)", prod_sorted(kAddFrom, idn), add_b},
      {"add  sorted prod sorted (wave)", prod_sorted(kAddFrom, srt), add_b},
      {"add  sorted wave8 ntld+st /3", wvar(kAddFrom, srt, 8, true, true, 3), add_b},
      {"gath rand   prod (wave /8)", rowop(kAssignTo, rnd), gat_b},
      {"gath rand   wave /4", gath(rnd, 4), gat_b},
      {"gath rand   wave /8", gath(rnd, 8), gat_b},
      {"gath ident  prod (wave /8)", rowop(kAssignTo, idn), gat_b},
      {"gath ident  wave /4", gath(idn, 4), gat_b},
      {"init rand   prod (wave)", rowop(kInitFrom, rnd), init_b},
      {"init rand   wave8 ntst /4", wvar(kInitFrom, rnd, 8, false, true, 4), init_b},
      {"init ident  prod (wave)", rowop(kInitFrom, idn), init_b},
      {"init sorted prod (wave)", rowop(kInitFrom, srt), init_b},
      {"init sorted wave8 ntst /4", wvar(kInitFrom, srt, 8, false, true, 4), init_b},
      {"copy D2D 4 GiB", copy, 2.0 * n * 4},
  };
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  std::vector<std::vector<float>> ms(vs.size());
  for (auto &v : vs) v.f();  // warm-up
  CK(hipDeviceSynchronize());
  for (int r = 0; r < rounds; ++r)
    for (size_t i = 0; i < vs.size(); ++i) {
      CK(hipEventRecord(a, 0));
      vs[i].f();
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float t = 0;
      CK(hipEventElapsedTime(&t, a, b));
      ms[i].push_back(t);
    }
  CK(hipGetLastError());
  std::printf("%-28s %9s %9s %9s %8s\n", "variant", "med_ms", "min_ms", "TB/s", "%8TB/s");
  for (size_t i = 0; i < vs.size(); ++i) {
    auto m = ms[i];
    std::sort(m.begin(), m.end());
    const double med = m[m.size() / 2];
    const double tbs = vs[i].bytes / (med * 1e-3) / 1e12;
    std::printf("%-28s %9.4f %9.4f %9.3f %7.1f%%\n", vs[i].name.c_str(), med, m[0], tbs,
                100.0 * tbs / 8.0);
  }
  return 0;
}
