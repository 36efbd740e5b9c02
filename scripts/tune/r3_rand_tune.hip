// r3_rand_tune.hip — round-3 probe 4 (tuning harness, not product code; it
// #includes the product kernels): the box's ceiling for random-row traffic.
// The planned init / gather on a random index read 512-B source rows in random
// order and write the destination front to back (VERDICT r02 #6 asks >= 75 %
// of 8 TB/s; production is ~73 %).  This probe prices the access patterns
// alone, with one simple mover kernel (32 lanes x 16 B per 512-B row, RPG rows
// in flight per 32-lane group, 64-row tiles per wave, row ids from two uint32
// arrays), at block granularities of 512 B .. 4 KiB:
//   read    rows read in the given order, summed into a sink (read-only)
//   write   rows written in the given order (write-only)
//   copy    y[dst[i]] = x[src[i]]: gather (src random, dst sequential) and
//           scatter (src sequential, dst random)
// and the product's planned init / gather sorted by destination against the
// same ops sorted by source (sequential reads, random writes).  Every copy
// variant is bit-checked against the product's gather on the same pairs.
// Usage: r3_rand_tune [rounds]
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
__device__ float g_rand_sink[64];

// MODE 0 read, 1 write, 2 copy.  src/dst: 512-B row ids (dst unused for read,
// src unused for write).
template <int MODE, int RPG, bool NTL, bool NTS>
__global__ __launch_bounds__(kBlock) void mover_kernel(float *__restrict__ y, const float *__restrict__ x,
                                                       const uint32_t *__restrict__ src,
                                                       const uint32_t *__restrict__ dst, size_t num_rows) {
  typedef __attribute__((address_space(1))) f4 GT;
  constexpr int LPR = 32, kG = 2, kRowsPerGroup = 32;
  const int wl = threadIdx.x & 63, lane = wl % LPR, gw = wl / LPR;
  const size_t wave = ((size_t)blockIdx.x * kBlock + threadIdx.x) / 64;
  const size_t wstride = (size_t)gridDim.x * (kBlock / 64) * 64;
  f4 acc = f4(0.0f);
  for (size_t t = wave * 64; t < num_rows; t += wstride) {
    const bool live = t + wl < num_rows;
    const uint32_t ms = (MODE != 1 && live) ? src[t + wl] : 0u;
    const uint32_t md = (MODE != 0 && live) ? dst[t + wl] : 0u;
    const size_t rows_here = num_rows - t < 64 ? num_rows - t : 64;
    for (int i0 = 0; i0 < kRowsPerGroup; i0 += RPG) {
      f4 xs[RPG];
      if (MODE != 1) {
#pragma unroll
        for (int k = 0; k < RPG; ++k) {
          const int rt = gw + kG * (i0 + k);
          const uint32_t s = __shfl(ms, rt);
          if ((size_t)rt < rows_here) {
            const GT *p = reinterpret_cast<const GT *>(reinterpret_cast<uint64_t>(x + (size_t)s * W)) + lane;
            xs[k] = NTL ? __builtin_nontemporal_load(p) : *p;
          }
        }
      }
      if (MODE == 0) {
#pragma unroll
        for (int k = 0; k < RPG; ++k) acc += xs[k];
      } else {
#pragma unroll
        for (int k = 0; k < RPG; ++k) {
          const int rt = gw + kG * (i0 + k);
          const uint32_t d = __shfl(md, rt);
          if ((size_t)rt < rows_here) {
            GT *p = reinterpret_cast<GT *>(reinterpret_cast<uint64_t>(y + (size_t)d * W)) + lane;
            const f4 v = MODE == 2 ? xs[k] : f4((float)rt);
            if (NTS)
              __builtin_nontemporal_store(v, p);
            else
              *p = v;
          }
        }
      }
    }
  }
  if (MODE == 0 && acc.x + acc.y + acc.z + acc.w == -1234.5f) g_rand_sink[blockIdx.x % 64] = acc.x;
}

__global__ void mismatch_kernel(const uint32_t *a, const uint32_t *b, size_t n, unsigned long long *cnt) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  unsigned long long c = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) c += a[i] != b[i];
  if (c) atomicAdd(cnt, c);
}

template <int MODE, int RPG, bool NTL, bool NTS>
int resident() {
  static std::atomic<int> occ{0};
  return resident_blocks(reinterpret_cast<const void *>(&mover_kernel<MODE, RPG, NTL, NTS>), occ);
}

// row ids in block-permuted order: blocks of `gran` consecutive 512-B rows,
// the blocks in a random permutation (gran == 0: identity)
static std::vector<uint32_t> block_perm(size_t gran, std::mt19937_64 &g) {
  std::vector<uint32_t> ids(R);
  if (gran == 0) {
    std::iota(ids.begin(), ids.end(), 0u);
    return ids;
  }
  std::vector<uint32_t> b(R / gran);
  std::iota(b.begin(), b.end(), 0u);
  std::shuffle(b.begin(), b.end(), g);
  for (size_t i = 0; i < b.size(); ++i)
    for (size_t j = 0; j < gran; ++j) ids[i * gran + j] = (uint32_t)(b[i] * gran + j);
  return ids;
}

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 5;
  std::mt19937_64 g(4);
  const std::vector<uint32_t> seq = block_perm(0, g);
  const size_t grans[] = {1, 2, 4, 8};
  std::vector<std::vector<uint32_t>> perms;
  for (size_t gr : grans) perms.push_back(block_perm(gr, g));
  uint32_t *dseq, *dperm[4];
  CK(hipMalloc(&dseq, R * 4));
  CK(hipMemcpy(dseq, seq.data(), R * 4, hipMemcpyHostToDevice));
  for (int i = 0; i < 4; ++i) {
    CK(hipMalloc(&dperm[i], R * 4));
    CK(hipMemcpy(dperm[i], perms[i].data(), R * 4, hipMemcpyHostToDevice));
  }
  // product-format indices for the 512-B random permutation p = perms[0]:
  // gather y[id0] = x[id1]: dst-sorted {i, p[i]}; src-sorted {q[j], j} (q = p^-1)
  // init (scatter) y[id1] = 0 + x[id0] with y[p[i]] = x[i]: dst-sorted {q[d], d};
  // src-sorted {i, p[i]}
  const std::vector<uint32_t> &p = perms[0];
  std::vector<uint32_t> q(R);
  for (size_t i = 0; i < R; ++i) q[p[i]] = (uint32_t)i;
  std::vector<gp_double_index> gd(R), gs(R), id_(R), is(R);
  for (size_t i = 0; i < R; ++i) {
    gd[i] = {i, p[i]};
    gs[i] = {q[i], i};
    id_[i] = {q[i], i};
    is[i] = {i, p[i]};
  }
  gp_double_index *igd, *igs, *iid, *iis;
  for (auto pr : {std::make_pair(&igd, &gd), std::make_pair(&igs, &gs), std::make_pair(&iid, &id_),
                  std::make_pair(&iis, &is)}) {
    CK(hipMalloc(pr.first, R * 16));
    CK(hipMemcpy(*pr.first, pr.second->data(), R * 16, hipMemcpyHostToDevice));
  }
  unsigned long long *cnt;
  CK(hipMalloc(&cnt, 8));
  const size_t G = (size_t)num_cus();
  hipEvent_t ea, eb;
  CK(hipEventCreate(&ea));
  CK(hipEventCreate(&eb));

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
    double bytes;
    int check;  // 0 none; 1 gather on perms[0] (y[i] = x[p[i]]); 2 scatter (y[p[i]] = x[i])
  };
  std::vector<V> vs;
  const double row = (double)W * 4;
#define MOV(MODE, RPGV, NTLV, NTSV, PCU, S, D, NAME, BYTES, CHK)                                        \
  vs.push_back({NAME,                                                                                   \
                [=] {                                                                                   \
                  const int occ = resident<MODE, RPGV, NTLV, NTSV>();                                   \
                  const size_t cap = G * (PCU > 0 ? PCU : occ);                                         \
                  const size_t grid = std::min((R + kBlock - 1) / kBlock, cap);                         \
                  hipLaunchKernelGGL((mover_kernel<MODE, RPGV, NTLV, NTSV>), dim3((unsigned)grid),      \
                                     dim3(kBlock), 0, 0, y, x, S, D, R);                                \
                },                                                                                      \
                BYTES, CHK});
  const double rb = R * row + 4.0 * R, cb = 2.0 * R * row + 8.0 * R;
  MOV(0, 8, true, true, 0, dseq, dseq, "read  seq          rpg8", rb, 0)
  MOV(0, 16, true, true, 0, dseq, dseq, "read  seq          rpg16", rb, 0)
  MOV(0, 8, true, true, 0, dperm[0], dseq, "read  rand 512B    rpg8", rb, 0)
  MOV(0, 16, true, true, 0, dperm[0], dseq, "read  rand 512B    rpg16", rb, 0)
  MOV(0, 32, true, true, 0, dperm[0], dseq, "read  rand 512B    rpg32", rb, 0)
  MOV(0, 16, false, true, 0, dperm[0], dseq, "read  rand 512B pl rpg16", rb, 0)
  MOV(0, 16, true, true, 0, dperm[1], dseq, "read  rand 1K      rpg16", rb, 0)
  MOV(0, 16, true, true, 0, dperm[2], dseq, "read  rand 2K      rpg16", rb, 0)
  MOV(0, 16, true, true, 0, dperm[3], dseq, "read  rand 4K      rpg16", rb, 0)
  MOV(1, 8, true, true, 0, dseq, dseq, "write seq          rpg8", rb, 0)
  MOV(1, 8, true, true, 0, dseq, dperm[0], "write rand 512B    rpg8", rb, 0)
  MOV(1, 16, true, true, 0, dseq, dperm[0], "write rand 512B    rpg16", rb, 0)
  MOV(1, 8, true, false, 0, dseq, dperm[0], "write rand 512B pl rpg8", rb, 0)
  MOV(1, 8, true, true, 0, dseq, dperm[1], "write rand 1K      rpg8", rb, 0)
  MOV(1, 8, true, true, 0, dseq, dperm[2], "write rand 2K      rpg8", rb, 0)
  MOV(1, 8, true, true, 0, dseq, dperm[3], "write rand 4K      rpg8", rb, 0)
  MOV(2, 8, true, true, 0, dseq, dseq, "copy  seq->seq     rpg8", cb, 0)
  MOV(2, 8, true, true, 0, dperm[0], dseq, "gath  rand->seq    rpg8", cb, 1)
  MOV(2, 16, true, true, 0, dperm[0], dseq, "gath  rand->seq    rpg16", cb, 1)
  MOV(2, 8, true, true, 0, dseq, dperm[0], "scat  seq->rand    rpg8", cb, 2)
  MOV(2, 16, true, true, 0, dseq, dperm[0], "scat  seq->rand    rpg16", cb, 2)
  MOV(2, 8, true, false, 0, dseq, dperm[0], "scat  seq->rand pl rpg8", cb, 2)
  MOV(2, 8, true, true, 0, dperm[1], dseq, "gath  rand1K->seq  rpg8", cb, 0)
  MOV(2, 8, true, true, 0, dseq, dperm[1], "scat  seq->rand1K  rpg8", cb, 0)
  MOV(2, 8, true, true, 0, dperm[3], dseq, "gath  rand4K->seq  rpg8", cb, 0)
  MOV(2, 8, true, true, 0, dseq, dperm[3], "scat  seq->rand4K  rpg8", cb, 0)
#undef MOV
  const double pb = 2.0 * R * row + 16.0 * R;
  vs.push_back({"prod gather dst-sorted", [&] { launch_row_op<kAssignTo>(y, x, igd, R, {0, 0}, W, ~size_t(0), 0, true); }, pb, 1});
  vs.push_back({"prod gather src-sorted", [&] { launch_row_op<kAssignTo>(y, x, igs, R, {0, 0}, W, ~size_t(0), 0, true); }, pb, 1});
  vs.push_back({"prod init   dst-sorted", [&] { launch_row_op<kInitFrom>(y, x, iid, R, {0, 0}, W, ~size_t(0), 0, true); }, pb, 2});
  vs.push_back({"prod init   src-sorted", [&] { launch_row_op<kInitFrom>(y, x, iis, R, {0, 0}, W, ~size_t(0), 0, true); }, pb, 2});

  // references: 1 gather y[i] = x[p[i]] (prod gather on gd), 2 scatter y[p[i]] = x[i] (prod init on iid)
  for (int c = 1; c <= 2; ++c) {
    if (c == 1)
      launch_row_op<kAssignTo>(yr, x, igd, R, {0, 0}, W, ~size_t(0), 0, true);
    else
      launch_row_op<kInitFrom>(yr, x, iid, R, {0, 0}, W, ~size_t(0), 0, true);
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
  std::printf("8M rows x 512 B; bytes = rows moved (+ index)\n");
  std::printf("%-28s %9s %9s %8s\n", "variant", "med_ms", "min_ms", "%8TB/s");
  for (size_t i = 0; i < vs.size(); ++i) {
    auto m = ms[i];
    std::sort(m.begin(), m.end());
    const double med = m[m.size() / 2];
    std::printf("%-28s %9.4f %9.4f %7.1f%%\n", vs[i].name.c_str(), med, m[0], 100.0 * vs[i].bytes / (med * 1e-3) / 8e12);
  }
  return 0;
}
