// r3_row_tune2.hip — round-3 probe, second pass (tuning harness, not product
// code; it #includes the product kernels).
//
// Pass 1 (r3_row_tune.hip, profiles/r03/tune/r3_row_tune.txt) found: binning
// the op-order scatter-add by destination needs windows of ~64 rows before it
// pays (bin6 70.9 % vs 66.0 %; bin12 67.6 %) and a counting sort costs 0.14-
// 0.28 ms; the indexed sweep loses to the wave map on sorted residuals; the
// index scan ran at 1.9 TB/s.  Here:
//  1. the production index scan (17 loads in flight per wave) + D2H + sync;
//  2. a full device sort of the (destination, source) pairs by hipCUB's radix
//     sort (rocPRIM onesweep), 23 key bits, u32 keys and values: is it cheap
//     enough to turn the op-order add into the destination-sorted one?
//  3. the row kernels on physically contiguous buffers (what libgeeps'
//     gp_malloc_device returns for big buffers) against plain hipMalloc:
//     op-order add, sorted add / init, random gather, identity sweep.
// Usage: r3_row_tune2 [rounds]
#include "../../geeps_amd/csrc/gp_reduce.hip"

#include <hipcub/hipcub.hpp>

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

__global__ void split_kernel(const gp_double_index *__restrict__ idx, size_t n, uint32_t *__restrict__ key,
                             uint32_t *__restrict__ val) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const gp_double_index e = idx[i];
    key[i] = (uint32_t)e.id1;
    val[i] = (uint32_t)e.id0;
  }
}

__global__ void join_kernel(const uint32_t *__restrict__ key, const uint32_t *__restrict__ val, size_t n,
                            gp_double_index *__restrict__ out) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    out[i] = gp_double_index{val[i], key[i]};
}

__global__ void mismatch_kernel(const uint32_t *a, const uint32_t *b, size_t n, unsigned long long *cnt) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  unsigned long long c = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) c += a[i] != b[i];
  if (c) atomicAdd(cnt, c);
}

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 5;
  float *x, *y, *xc, *yc;
  CK(hipMalloc(&x, N * 4));
  CK(hipMalloc(&y, N * 4));
  CK(hipExtMallocWithFlags(reinterpret_cast<void **>(&xc), N * 4, hipDeviceMallocContiguous));
  CK(hipExtMallocWithFlags(reinterpret_cast<void **>(&yc), N * 4, hipDeviceMallocContiguous));
  std::mt19937_64 g(3);
  std::vector<uint64_t> perm(R);
  std::iota(perm.begin(), perm.end(), 0);
  std::shuffle(perm.begin(), perm.end(), g);
  {
    std::vector<float> h(N);
    std::uniform_real_distribution<float> d(-0.5f, 0.5f);
    for (size_t i = 0; i < N; ++i) h[i] = d(g);
    CK(hipMemcpy(x, h.data(), N * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(xc, h.data(), N * 4, hipMemcpyHostToDevice));
    for (size_t i = 0; i < N; ++i) h[i] = d(g);
    CK(hipMemcpy(y, h.data(), N * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(yc, h.data(), N * 4, hipMemcpyHostToDevice));
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
  gp_double_index *rnd = upload(a), *srt = upload(b), *idn = upload(c), *rnd_copy = upload(a), *sorted_out;
  CK(hipMalloc(&sorted_out, R * 16));
  uint32_t *k0, *v0, *k1, *v1;
  CK(hipMalloc(&k0, R * 4));
  CK(hipMalloc(&v0, R * 4));
  CK(hipMalloc(&k1, R * 4));
  CK(hipMalloc(&v1, R * 4));
  size_t temp_bytes = 0;
  CK(hipcub::DeviceRadixSort::SortPairs(nullptr, temp_bytes, k0, k1, v0, v1, (int)R, 0, 23, 0));
  void *temp;
  CK(hipMalloc(&temp, temp_bytes));
  std::printf("hipcub temp bytes %zu\n", temp_bytes);
  char *ws, *hws;
  const size_t groups = (R / 64 + kScanGroupTiles - 1) / kScanGroupTiles;
  const size_t scan_bytes = kScanWordsOff + groups * kScanWords * 8;
  CK(hipMalloc(&ws, scan_bytes));
  CK(hipHostMalloc(reinterpret_cast<void **>(&hws), scan_bytes, hipHostMallocDefault));
  const size_t G = (size_t)num_cus();
  auto scan = [&](const gp_double_index *ix, bool d2h, bool cmp = false, const gp_double_index *cmp_against = nullptr) {
    if (!cmp_against) cmp_against = idn;
    return [=] {
      CK(hipMemsetAsync(ws, 0, sizeof(ScanHeader), 0));
      if (cmp)
        hipLaunchKernelGGL((index_scan_kernel<kAddFrom, true>), dim3((unsigned)std::min(groups, G * 8)),
                           dim3(kBlock), 0, 0, ix, R, 0, 0, W, ~size_t(0), cmp_against, ws);
      else
        hipLaunchKernelGGL((index_scan_kernel<kAddFrom, false>), dim3((unsigned)std::min(groups, G * 8)),
                           dim3(kBlock), 0, 0, ix, R, 0, 0, W, ~size_t(0), nullptr, ws);
      if (d2h) {
        CK(hipMemcpyAsync(hws, ws, scan_bytes, hipMemcpyDeviceToHost, 0));
        CK(hipStreamSynchronize(0));
      }
    };
  };
  auto sort = [&](int part) {  // 1 split, 2 + sort, 3 + join
    return [=] {
      size_t tb = temp_bytes;
      hipLaunchKernelGGL(split_kernel, dim3((unsigned)(G * 8)), dim3(256), 0, 0, rnd, R, k0, v0);
      if (part >= 2) CK(hipcub::DeviceRadixSort::SortPairs(temp, tb, k0, k1, v0, v1, (int)R, 0, 23, 0));
      if (part >= 3) hipLaunchKernelGGL(join_kernel, dim3((unsigned)(G * 8)), dim3(256), 0, 0, k1, v1, R, sorted_out);
    };
  };
  auto add = [&](float *yy, float *xx, const gp_double_index *ix, bool sorted) {
    return [=] { launch_row_op<kAddFrom>(yy, xx, ix, R, {0, 0}, W, ~size_t(0), 0, sorted); };
  };
  auto init = [&](float *yy, float *xx, const gp_double_index *ix) {
    return [=] { launch_row_op<kInitFrom>(yy, xx, ix, R, {0, 0}, W, ~size_t(0), 0, true); };
  };
  auto gath = [&](float *yy, float *xx, const gp_double_index *ix) {
    return [=] { launch_row_op<kAssignTo>(yy, xx, ix, R, {0, 0}, W, ~size_t(0), 0, true); };
  };
  auto dense = [&](float *yy, float *xx) {
    return [=] {
      BucketPtrs bp = {};
      bp.p[0] = xx;
      launch_bucket_sum_nb<1>(yy, yy, bp, N, 0);
    };
  };
  const double add_b = 3.0 * N * 4 + 16.0 * R, one_b = 2.0 * N * 4 + 16.0 * R;
  struct V {
    std::string name;
    std::function<void()> f;
    double bytes;
  };
  std::vector<V> vs = {
      {"scan (prod v2)", scan(rnd, false), 16.0 * R},
      {"scan + D2H + sync", scan(rnd, true), 16.0 * R},
      {"scan ident + D2H + sync", scan(idn, true), 16.0 * R},
      {"scan + compare, all differ", scan(rnd, false, true), 32.0 * R},
      {"scan + compare, equal (kernel)", scan(rnd, false, true, rnd_copy), 32.0 * R},
      {"scan + compare, equal + D2H + sync", scan(rnd, true, true, rnd_copy), 32.0 * R},
      {"sort: split", sort(1), 24.0 * R},
      {"sort: split + radix 23b", sort(2), 24.0 * R},
      {"sort: split + radix + join", sort(3), 24.0 * R},
      {"add  rand  row_op  plain", add(y, x, rnd, false), add_b},
      {"add  rand  row_op  contig", add(yc, xc, rnd, false), add_b},
      {"add  sorted wave   plain", add(y, x, srt, true), add_b},
      {"add  sorted wave   contig", add(yc, xc, srt, true), add_b},
      {"add  devsorted wave plain", add(y, x, sorted_out, true), add_b},
      {"add  ident dense   plain", dense(y, x), 3.0 * N * 4},
      {"add  ident dense   contig", dense(yc, xc), 3.0 * N * 4},
      {"init rand  wave    plain", [=] { launch_row_op<kInitFrom>(y, x, rnd, R, {0, 0}, W, ~size_t(0), 0); }, one_b},
      {"init rand  wave    contig", [=] { launch_row_op<kInitFrom>(yc, xc, rnd, R, {0, 0}, W, ~size_t(0), 0); }, one_b},
      {"init sorted wave   plain", init(y, x, srt), one_b},
      {"init sorted wave   contig", init(yc, xc, srt), one_b},
      {"gath rand  wave    plain", gath(y, x, rnd), one_b},
      {"gath rand  wave    contig", gath(yc, xc, rnd), one_b},
  };
  // checks: the device sort is the host sort; the add through it matches
  sort(3)();
  {
    std::vector<gp_double_index> h(R);
    CK(hipMemcpy(h.data(), sorted_out, R * 16, hipMemcpyDeviceToHost));
    bool ok = true;
    for (size_t r = 0; r < R && ok; ++r) ok = h[r].id1 == r && h[r].id0 == b[r].id0;
    std::printf("check device sort %s\n", ok ? "ok" : "FAILED");
    if (!ok) return 3;
    scan(idn, true)();
    const ScanHeader *hd = reinterpret_cast<const ScanHeader *>(hws);
    const uint64_t *w = reinterpret_cast<const uint64_t *>(hws + kScanWordsOff);
    std::printf("check scan ident: starts %u max %llu words %llx %llx %llx\n", hd->n_starts,
                (unsigned long long)w[3], (unsigned long long)w[0], (unsigned long long)w[1],
                (unsigned long long)w[2]);
    scan(rnd, true, true)();
    std::printf("check scan rand vs ident copy: starts %u mismatching waves %u max %llu\n", hd->n_starts,
                hd->mismatches, (unsigned long long)w[3]);
  }
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
