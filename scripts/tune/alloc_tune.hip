// alloc_tune.hip — does the allocation KIND fix the 8-way bucket sum's
// per-allocation spread (placement_tune.hip)?  (tuning harness, not product
// code; it #includes the product kernels)
//
// On ONE box, interleaved rounds of the production launch over 36-GiB arenas
// (8 buckets + master, master last) from plain hipMalloc, from
// hipExtMallocWithFlags(hipDeviceMallocContiguous), and from a window 1 GiB
// into a larger hipMalloc.  Usage: alloc_tune [rounds]
#include "../../geeps_amd/csrc/gp_reduce.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
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

constexpr size_t kN = (1ull << 20) * 1024;  // floats per buffer (4 GiB)

__global__ void fill_k(float *p, size_t n, unsigned seed) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    unsigned x = (unsigned)(i * 2654435761u) ^ seed;
    x ^= x >> 13;
    x *= 0x5bd1e995u;
    x ^= x >> 15;
    p[i] = (float)(x & 0xffffff) / 16777216.0f - 0.5f;
  }
}



// Diagnostics per arena: the nine read streams alone (no store), and the
// master's write stream alone.
__global__ __launch_bounds__(kBlock) void read9(const f4 *__restrict__ m, BucketPtrs b, size_t n4,
                                                f4 *__restrict__ sink, int flag) {
  constexpr int U = 4;
  const size_t tile = (size_t)kBlock * U;
  const size_t stride = (size_t)gridDim.x * tile;
  f4 tot = {0, 0, 0, 0};
  for (size_t base = (size_t)blockIdx.x * tile + threadIdx.x; base + (U - 1) * kBlock < n4;
       base += stride) {
    f4 v[9][U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[8][u] = m[base + u * kBlock];
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int u = 0; u < U; ++u)
        v[k][u] = __builtin_nontemporal_load(reinterpret_cast<const f4 *>(b.p[k]) + base + u * kBlock);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int k = 0; k < 9; ++k) tot += v[k][u];
  }
  if (flag) sink[blockIdx.x * kBlock + threadIdx.x] = tot;
}

__global__ __launch_bounds__(kBlock) void write1(f4 *__restrict__ m, size_t n4) {
  const size_t stride = (size_t)gridDim.x * kBlock;
  const f4 z = {1, 2, 3, 4};
  for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n4; i += stride) m[i] = z;
}

struct Set {
  std::string name;
  BucketPtrs b;
  float *master;
};

Set carve(const std::string &name, char *a) {
  Set s{name, {}, nullptr};
  for (int k = 0; k < 8; ++k) {
    s.b.p[k] = reinterpret_cast<const float *>(a + (size_t)k * kN * 4);
    fill_k<<<4096, 256>>>(reinterpret_cast<float *>(a + (size_t)k * kN * 4), kN, 1000 + k);
  }
  s.master = reinterpret_cast<float *>(a + (size_t)8 * kN * 4);
  fill_k<<<4096, 256>>>(s.master, kN, 77);
  CK(hipDeviceSynchronize());
  return s;
}

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 5;
  const size_t bytes = 9 * kN * 4;
  std::vector<Set> sets;
  for (int i = 0; i < 3; ++i) {
    char *a = nullptr;
    CK(hipMalloc(&a, bytes));
    sets.push_back(carve("hipMalloc #" + std::to_string(i + 1), a));
  }
  for (int i = 0; i < 2; ++i) {
    char *a = nullptr;
    hipError_t e = hipExtMallocWithFlags(reinterpret_cast<void **>(&a), bytes, hipDeviceMallocContiguous);
    if (e != hipSuccess) {
      std::printf("contiguous #%d: %s\n", i + 1, hipGetErrorString(e));
      (void)hipGetLastError();
      continue;
    }
    sets.push_back(carve("contiguous #" + std::to_string(i + 1), a));
  }
  {
    char *a = nullptr;
    CK(hipMalloc(&a, bytes + (4ull << 30)));
    sets.push_back(carve("hipMalloc +1GiB window", a + (1ull << 30)));
  }
  struct V {
    std::string name;
    std::function<void()> run;
    std::vector<float> ms;
  };
  std::vector<V> vs;
  const unsigned grid2 = (unsigned)num_cus() * 2, grid8 = (unsigned)num_cus() * 8;
  std::vector<double> vbytes;
  for (auto &s : sets) {
    std::vector<const float *> bv(s.b.p, s.b.p + 8);
    float *m = s.master;
    BucketPtrs bp = s.b;
    vs.push_back(V{s.name + " sum", [=]() { gp_bucket_sum_apply(m, bv.data(), 8, kN, nullptr); }, {}});
    vbytes.push_back(10.0 * kN * 4);
    vs.push_back(V{s.name + " read9", [=]() { read9<<<grid2, kBlock>>>(reinterpret_cast<const f4 *>(m), bp, kN / 4, reinterpret_cast<f4 *>(m), 0); }, {}});
    vbytes.push_back(9.0 * kN * 4);
    vs.push_back(V{s.name + " write1", [=]() { write1<<<grid8, kBlock>>>(reinterpret_cast<f4 *>(m), kN / 4); }, {}});
    vbytes.push_back(1.0 * kN * 4);
  }
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
  }
  std::printf("%-34s %10s %10s %10s %8s\n", "allocation / kernel", "med_ms", "min_ms", "GB/s", "frac8T");
  for (size_t i = 0; i < vs.size(); ++i) {
    auto &v = vs[i];
    const double sum_b = vbytes[i];
    std::sort(v.ms.begin(), v.ms.end());
    const double med = v.ms[v.ms.size() / 2];
    const double gbs = sum_b / (med * 1e-3) / 1e9;
    std::printf("%-34s %10.4f %10.4f %10.1f %8.4f\n", v.name.c_str(), med, v.ms[0], gbs, gbs / 8000.0);
  }
  return 0;
}
