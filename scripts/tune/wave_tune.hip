// wave_tune.hip — rows in flight for the wave-map row kernel on a row plan's
// residual (tuning harness, not product code; it #includes the product
// kernels).  The 8-way sweep sum gained 2-3.5 % from fewer loads in flight per
// wave (bursts of 2 tiles: a narrower window of outstanding addresses,
// big_tune.hip).  Here the same question for row_wave_kernel, which production
// launches as one resident round of blocks (CUs x blocks resident per CU) with
// 8 rows per 32-lane group in flight: 8 M rows of 128 floats, a random
// permutation index in destination order (what a scatter plan's residual and
// a gather plan's residual hold), scatter-add, fused init and gather, with 4 or
// 8 rows per group and 1, 2 or the resident count of blocks per CU.  Each
// variant is bit-checked against the production planned call.  Pass 1
// (profiles/r02/tune/wave_tune.txt): the scatter forms want every resident
// block (fewer lose 10-50 %); the gather ran +2.7 % at 2 blocks per CU against
// production's 4.  Pass 2: the gather at 2-4 blocks per CU, random and
// identity (the unplanned call's) indexes (wave_tune2.txt: within noise).
// Pass 3: the unplanned scatter-add (row_op_kernel, op order) at grid caps of
// 1-8 blocks per CU (wave_tune3{,b}.txt: 2 per CU +4 % identity, +0.3 %
// random; adopted).  Pass 4 (this version): the segmented forms at 2-8
// (wave_tune4{,b}.txt: the segmented add +5-7 % at 4 per CU, adopted; the
// segmented gather keeps 8).  Pass 5 (this version): rows per group x blocks
// per CU around the adopted flat scatter-add (4 rows, 2 per CU)
// (wave_tune5.txt: the adopted shape is best; 2 or 8 rows per group at 1-4
// blocks per CU lose 1.6-11 %).  Pass 6 (this version): the unplanned init
// and gather in op order, wave-map kernel against row_op_kernel at 1-8 per CU
// (wave_tune6{,b}.txt: the init +14 % identity / -3 % random at 2 per CU, but
// a net loss in the bench line, profiles/r02/rowinit/; the gather keeps the
// wave map).  Pass 7 (this version): the oplog side's cache policy for the
// op-order scatter-add at its new 2 blocks per CU (wave_tune7{,b}.txt: nt
// stores +0.7-1.2 % random / +1.5-2.2 % identity on two boxes, but the
// bench line's random leg lost 4-5 % with them (profiles/r02/ntst/): not
// adopted; nt loads lose on a random index).
// Usage: wave_tune [rounds]
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

__global__ void fill_k(float *p, size_t n, unsigned seed) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    unsigned v = (unsigned)(i * 2654435761u) ^ seed;
    v ^= v >> 13;
    v *= 0x5bd1e995u;
    v ^= v >> 15;
    p[i] = (float)(v & 0xffffff) / 16777216.0f - 0.5f;
  }
}

__global__ void diff_k(const unsigned *a, const unsigned *b, size_t n, unsigned long long *bad) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  unsigned long long c = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) c += a[i] != b[i];
  if (c) atomicAdd(bad, c);
}

// the unplanned scatter-add's kernel (row_op_kernel, op order) at a grid cap of
// per_cu blocks per CU (production: kBlocksPerCU = 8)
template <int OP, int RPG>
void rowop(float *y, const float *x, const gp_double_index *ix, int per_cu) {
  const size_t groups = (R + RPG - 1) / RPG;
  const size_t grid = std::min((groups + kBlock / 32 - 1) / (kBlock / 32), (size_t)num_cus() * per_cu);
  hipLaunchKernelGGL((row_op_kernel<f4, 4, OP, 32, RPG>), dim3((unsigned)grid), dim3(kBlock), 0, 0, y, x, ix, R,
                     0, 0, W, W / 4, ~size_t(0));
}

// the segmented forms (row_op_seg_kernel: Read's segmented gather residual,
// read-my-writes' segmented add) at a grid cap of per_cu blocks per CU
template <int OP, int SEG>
void rowseg(float *flat, const gp_row_segments &t, const gp_double_index *ix, int per_cu) {
  constexpr int RPG = OP == kAddFrom ? 4 : 8;
  const size_t groups = (R + RPG - 1) / RPG;
  const size_t grid = std::min((groups + kBlock / 32 - 1) / (kBlock / 32), (size_t)num_cus() * per_cu);
  SegArg<SEG> seg;
  seg.t = t;
  float *y = SEG == kSegX ? flat : nullptr;
  const float *x = SEG == kSegY ? flat : nullptr;
  hipLaunchKernelGGL((row_op_seg_kernel<f4, 4, OP, 32, RPG, SEG>), dim3((unsigned)grid), dim3(kBlock), 0, 0, y, x,
                     ix, R, 0, 0, W, W / 4, ~size_t(0), seg);
}


// row_op_kernel's whole-row path with the oplog (y) side's cache policy as a
// parameter: YL non-temporal y loads, YS non-temporal y stores (production:
// plain both; the op buffer x is read non-temporally either way)
template <int RPG, bool YL, bool YS>
__global__ __launch_bounds__(kBlock) void add_var_kernel(float *__restrict__ y, const float *__restrict__ x,
                                                         const gp_double_index *__restrict__ index,
                                                         size_t num_rows, size_t vw) {
  constexpr int LPR = 32, kGroups = kBlock / LPR;
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
#pragma unroll
      for (int k = 0; k < RPG; ++k)
        if (live[k]) ys[k] = YL ? __builtin_nontemporal_load(yv + to[k] * vw + j) : yv[to[k] * vw + j];
#pragma unroll
      for (int k = 0; k < RPG; ++k)
        if (live[k]) {
          if (YS)
            __builtin_nontemporal_store(ys[k] + xs[k], yv + to[k] * vw + j);
          else
            yv[to[k] * vw + j] = ys[k] + xs[k];
        }
    }
  }
}

template <bool YL, bool YS>
void addvar(float *y, const float *x, const gp_double_index *ix, int per_cu) {
  const size_t groups = (R + 3) / 4;
  const size_t grid = std::min((groups + kBlock / 32 - 1) / (kBlock / 32), (size_t)num_cus() * per_cu);
  hipLaunchKernelGGL((add_var_kernel<4, YL, YS>), dim3((unsigned)grid), dim3(kBlock), 0, 0, y, x, ix, R, W / 4);
}

template <int OP, int RPG>
int occupancy() {
  int occ = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
      &occ, reinterpret_cast<const void *>(&row_wave_kernel<f4, OP, 32, RPG, kFlat>), kBlock, 0));
  return occ;
}

// y (+)= x / y = x over the sorted index: rows [0, R) through row_wave_kernel
template <int OP, int RPG>
void wave(float *y, const float *x, const gp_double_index *ix, int per_cu) {
  const size_t grid = std::min((R + kBlock - 1) / kBlock, (size_t)num_cus() * per_cu);
  const SegArg<kFlat> flat{};
  hipLaunchKernelGGL((row_wave_kernel<f4, OP, 32, RPG, kFlat>), dim3((unsigned)grid), dim3(kBlock), 0, 0, y,
                     x, ix, R, 0, 0, W, W / 4, ~size_t(0), flat);
}

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 7;
  float *x, *y, *y0, *ref;
  unsigned long long *bad;
  CK(hipMalloc(&x, N * 4));
  CK(hipMalloc(&y, N * 4));
  CK(hipMalloc(&y0, N * 4));
  CK(hipMalloc(&ref, N * 4));
  CK(hipMalloc(&bad, 8));
  fill_k<<<4096, 256>>>(x, N, 11);
  fill_k<<<4096, 256>>>(y0, N, 22);
  // random permutation: scatter index (id0 = op row, id1 = cache row) sorted by
  // id1; gather index (id0 = op row, id1 = cache row) sorted by id0 (= op order)
  std::vector<uint64_t> perm(R);
  std::iota(perm.begin(), perm.end(), 0);
  std::mt19937_64 rng(7);
  std::shuffle(perm.begin(), perm.end(), rng);
  std::vector<gp_double_index> sidx(R), gidx(R);
  for (size_t r = 0; r < R; ++r) {
    sidx[perm[r]] = gp_double_index{r, perm[r]};  // position perm[r]: ascending id1
    gidx[r] = gp_double_index{r, perm[r]};
  }
  gp_double_index *ds, *dg;
  CK(hipMalloc(&ds, R * 16));
  CK(hipMalloc(&dg, R * 16));
  CK(hipMemcpy(ds, sidx.data(), R * 16, hipMemcpyHostToDevice));
  CK(hipMemcpy(dg, gidx.data(), R * 16, hipMemcpyHostToDevice));
  gp_double_index *di;  // identity
  CK(hipMalloc(&di, R * 16));
  for (size_t r = 0; r < R; ++r) gidx[r] = gp_double_index{r, r};
  CK(hipMemcpy(di, gidx.data(), R * 16, hipMemcpyHostToDevice));
  for (size_t r = 0; r < R; ++r) gidx[r] = gp_double_index{r, perm[r]};
  gp_row_plan sp = nullptr, gp = nullptr;
  CK(gp_row_plan_create(&sp, sidx.data(), R, gp_double_index{0, 0}, W, ~size_t(0)) == 0 ? hipSuccess
                                                                                         : hipErrorUnknown);
  CK(gp_gather_plan_create(&gp, gidx.data(), R, gp_double_index{0, 0}, W, ~size_t(0)) == 0
         ? hipSuccess
         : hipErrorUnknown);
  std::printf("occupancy (blocks per CU): add R8 %d R4 %d, init R8 %d R4 %d, gather R8 %d R4 %d\n",
              occupancy<kAddFrom, 8>(), occupancy<kAddFrom, 4>(), occupancy<kInitFrom, 8>(),
              occupancy<kInitFrom, 4>(), occupancy<kAssignTo, 8>(), occupancy<kAssignTo, 4>());

  struct V {
    std::string name;
    int op;  // 0 add, 3 init, 1 gather
    std::function<void()> f;
    double bytes;
  };
  const double add_b = 3.0 * N * 4, two_b = 2.0 * N * 4;
  // gather: y[id0] = x[id1] -> x is the cache (read randomly), y the op buffer
  std::vector<V> vs;
  auto add_v = [&](const char *nm, std::function<void()> f) { vs.push_back({nm, 0, f, add_b}); };
  auto ini_v = [&](const char *nm, std::function<void()> f) { vs.push_back({nm, 3, f, two_b}); };
  auto gat_v = [&](const char *nm, std::function<void()> f) { vs.push_back({nm, 1, f, two_b}); };
  // op order: random (x sequential, y random) and identity
  std::vector<gp_double_index> ridx(R);
  for (size_t r = 0; r < R; ++r) ridx[r] = gp_double_index{r, perm[r]};
  gp_double_index *dr;
  CK(hipMalloc(&dr, R * 16));
  CK(hipMemcpy(dr, ridx.data(), R * 16, hipMemcpyHostToDevice));
  add_v("add rand prod (plain y, /2)", [=] { gp_scatter_add_rows(y, x, dr, R, gp_double_index{0, 0}, W, ~size_t(0), nullptr); });
  add_v("add rand var plain /2", [=] { addvar<false, false>(y, x, dr, 2); });
  add_v("add rand var nt ld+st /2", [=] { addvar<true, true>(y, x, dr, 2); });
  add_v("add rand var nt st /2", [=] { addvar<false, true>(y, x, dr, 2); });
  add_v("add rand var nt ld /2", [=] { addvar<true, false>(y, x, dr, 2); });
  add_v("add ident prod (plain y, /2)", [=] { gp_scatter_add_rows(y, x, di, R, gp_double_index{0, 0}, W, ~size_t(0), nullptr); });
  add_v("add ident var plain /2", [=] { addvar<false, false>(y, x, di, 2); });
  add_v("add ident var nt ld+st /2", [=] { addvar<true, true>(y, x, di, 2); });
  add_v("add ident var nt st /2", [=] { addvar<false, true>(y, x, di, 2); });
  add_v("add ident var nt ld /2", [=] { addvar<true, false>(y, x, di, 2); });
  // bit check against the production planned call of the same op
  for (size_t i = 0; i < vs.size(); ++i) {
    CK(hipMemcpy(y, y0, N * 4, hipMemcpyDeviceToDevice));
    vs[i].f();
    CK(hipDeviceSynchronize());
    if (vs[i].name.find("prod") != std::string::npos) {
      CK(hipMemcpy(ref, y, N * 4, hipMemcpyDeviceToDevice));
      continue;
    }
    CK(hipMemset(bad, 0, 8));
    diff_k<<<4096, 256>>>(reinterpret_cast<const unsigned *>(ref), reinterpret_cast<const unsigned *>(y), N, bad);
    unsigned long long hb = 0;
    CK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
    std::printf("%-22s vs prod: %llu mismatches\n", vs[i].name.c_str(), hb);
  }
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  std::vector<std::vector<float>> ms(vs.size());
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
  std::printf("%-22s %9s %9s %9s %8s\n", "variant", "med_ms", "min_ms", "TB/s", "%8TB/s");
  for (size_t i = 0; i < vs.size(); ++i) {
    auto m = ms[i];
    std::sort(m.begin(), m.end());
    const double med = m[m.size() / 2];
    const double tbs = vs[i].bytes / (med * 1e-3) / 1e12;
    std::printf("%-22s %9.4f %9.4f %9.3f %7.1f%%\n", vs[i].name.c_str(), med, m[0], tbs, 100.0 * tbs / 8.0);
  }
  gp_row_plan_destroy(sp);
  gp_row_plan_destroy(gp);
  return 0;
}
