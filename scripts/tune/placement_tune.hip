// placement_tune.hip — why does the same 8-way bucket sum take 7.2 ms on one
// MI355X box and 8.3 ms on another with the same copy rate?  (tuning harness,
// not product code; it #includes the product kernels)
//
// On ONE box, interleaved rounds of the production launch over several
// allocations of the same shape (does the time follow the allocation?), over
// padded arenas (does it follow the streams' relative offsets?), plus launch
// shapes that change how many pages are live at once, and read-only / copy
// ceilings.  Usage: placement_tune [rounds]
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

// Production loop, parameterised launch shape; optional XCD-contiguous tile
// remap (blocks b, b+8, ... run on one XCD: give each XCD a contiguous slice).
template <int U, bool XCD, bool STORE>
__global__ __launch_bounds__(kBlock) void bsum_shape(f4 *__restrict__ out, BucketPtrs b, size_t n4,
                                                     int flag) {
  constexpr int NB = 8;
  const size_t tile = (size_t)kBlock * U;
  const size_t stride = (size_t)gridDim.x * tile;
  unsigned lb = blockIdx.x;
  if (XCD) lb = (blockIdx.x % 8) * (gridDim.x / 8) + blockIdx.x / 8;
  f4 tot = {0, 0, 0, 0};
  size_t base = (size_t)lb * tile + threadIdx.x;
  for (; base + (U - 1) * kBlock < n4; base += stride) {
    f4 acc[U];
    f4 v[NB][U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = out[base + u * kBlock];
#pragma unroll
    for (int k = 0; k < NB; ++k)
#pragma unroll
      for (int u = 0; u < U; ++u)
        v[k][u] = __builtin_nontemporal_load(reinterpret_cast<const f4 *>(b.p[k]) + base + u * kBlock);
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int k = 0; k < NB; ++k) acc[u] += v[k][u];
      if (STORE)
        out[base + u * kBlock] = acc[u];
      else
        tot += acc[u];
    }
  }
  if (!STORE && flag) out[blockIdx.x * kBlock + threadIdx.x] = tot;
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

struct Set {
  std::string name;
  BucketPtrs b;
  float *master;
};

// 8 buckets then the master, buffer k at k * (kN*4 + pad) bytes in one allocation.
Set make_arena(const std::string &name, size_t pad) {
  char *a = nullptr;
  const size_t step = kN * 4 + pad;
  CK(hipMalloc(&a, 9 * step));
  Set s{name, {}, nullptr};
  for (int k = 0; k < 8; ++k) {
    s.b.p[k] = reinterpret_cast<const float *>(a + k * step);
    fill_k<<<4096, 256>>>(reinterpret_cast<float *>(a + k * step), kN, 1000 + k);
  }
  s.master = reinterpret_cast<float *>(a + 8 * step);
  fill_k<<<4096, 256>>>(s.master, kN, 77);
  CK(hipDeviceSynchronize());
  return s;
}

Set make_separate(const std::string &name) {
  Set s{name, {}, nullptr};
  for (int k = 0; k < 8; ++k) {
    float *p;
    CK(hipMalloc(&p, kN * 4));
    fill_k<<<4096, 256>>>(p, kN, 1000 + k);
    s.b.p[k] = p;
  }
  CK(hipMalloc(&s.master, kN * 4));
  fill_k<<<4096, 256>>>(s.master, kN, 77);
  CK(hipDeviceSynchronize());
  return s;
}

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 5;
  const size_t n4 = kN / 4;
  const int cus = num_cus();
  std::vector<Set> sets;
  sets.push_back(make_arena("arena#1 pad 0", 0));
  sets.push_back(make_arena("arena#2 pad 0", 0));
  sets.push_back(make_arena("arena#3 pad 0", 0));
  sets.push_back(make_arena("arena pad 2MiB", 2u << 20));
  sets.push_back(make_arena("arena pad 68KiB", 68u << 10));
  sets.push_back(make_separate("separate x9"));

  struct V {
    std::string name;
    double bytes;
    std::function<void()> run;
    std::vector<float> ms;
  };
  std::vector<V> vs;
  const double sum_b = 10.0 * kN * 4;
  for (auto &s : sets) {
    const float *bk[8];
    for (int k = 0; k < 8; ++k) bk[k] = s.b.p[k];
    std::vector<const float *> bv(bk, bk + 8);
    float *m = s.master;
    vs.push_back(V{"prod  " + s.name, sum_b, [=]() { gp_bucket_sum_apply(m, bv.data(), 8, kN, nullptr); }, {}});
  }
  const Set &a0 = sets[0];
  f4 *m0 = reinterpret_cast<f4 *>(a0.master);
  BucketPtrs b0 = a0.b;
  auto grid = [&](int per_cu) { return (unsigned)(cus * per_cu); };
  vs.push_back(V{"U1 pc8   arena#1", sum_b, [=]() { bsum_shape<1, false, true><<<grid(8), kBlock>>>(m0, b0, n4, 0); }, {}});
  vs.push_back(V{"U2 pc4   arena#1", sum_b, [=]() { bsum_shape<2, false, true><<<grid(4), kBlock>>>(m0, b0, n4, 0); }, {}});
  vs.push_back(V{"U4 pc2 XCD arena#1", sum_b, [=]() { bsum_shape<4, true, true><<<grid(2), kBlock>>>(m0, b0, n4, 0); }, {}});
  vs.push_back(V{"read9 U4 pc2 arena#1", 9.0 * kN * 4, [=]() { bsum_shape<4, false, false><<<grid(2), kBlock>>>(m0, b0, n4, 0); }, {}});
  f4 *dst = reinterpret_cast<f4 *>(sets[1].master);
  const f4 *src = reinterpret_cast<const f4 *>(a0.b.p[0]);
  vs.push_back(V{"copy 1R1W", 2.0 * kN * 4, [=]() { copy_k<<<grid(8), kBlock>>>(dst, src, n4); }, {}});

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
