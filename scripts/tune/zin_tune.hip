// zin_tune.hip — chunk shapes of the phase-separated sum's zero-input form
// (out = 0.0f + b0: a row plan's dense-run fused init), tuning harness, not
// product code (it #includes the product kernels).  4 GiB, 3 allocations,
// interleaved rounds, median.  Usage: zin_tune [rounds]
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

constexpr size_t kN = (size_t)1 << 30;  // floats (4 GiB)

template <int RT, bool ZIN>
void fixed_chunks(float *out, const float *x) {
  const size_t G = num_cus();
  const size_t n4 = kN / 4;
  const size_t tiles = n4 / kPhaseTile;
  const size_t chunk = G * (kPhaseLdsTiles + RT);
  PhasePlan p{RT, kPhaseLdsTiles + RT, RT > 0 ? 1 : 2, (tiles + chunk * (RT > 0 ? 1 : 2) - 1) / (chunk * (RT > 0 ? 1 : 2)), false};
  BucketPtrs b = {};
  b.p[0] = x;
  launch_phased<1, RT, false, ZIN>(out, ZIN ? nullptr : out, b, n4, p, 0);
}

// a plain streaming copy-with-add-of-zero, 4 strides in flight, no phases
__global__ __launch_bounds__(kBlock) void zin_stream(f4 *__restrict__ out, const f4 *__restrict__ in,
                                                     size_t n4) {
  const size_t tile = (size_t)kBlock * 4;
  const size_t stride = (size_t)gridDim.x * tile;
  for (size_t base = (size_t)blockIdx.x * tile + threadIdx.x; base + 3 * kBlock < n4; base += stride) {
    f4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(in + base + u * kBlock);
#pragma unroll
    for (int u = 0; u < 4; ++u) __builtin_nontemporal_store(f4(0.0f) + v[u], out + base + u * kBlock);
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

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 7;
  struct Buf {
    float *x, *y;
  };
  std::vector<Buf> bufs;
  std::vector<void *> spacers;
  for (int i = 0; i < 3; ++i) {
    void *sp = nullptr;
    CK(hipMalloc(&sp, (size_t)(1 + 700 * i) << 20));
    spacers.push_back(sp);
    Buf b;
    CK(hipMalloc(&b.x, kN * 4));
    CK(hipMalloc(&b.y, kN * 4));
    fill_k<<<4096, 256>>>(b.x, kN, 5 + i);
    bufs.push_back(b);
  }
  CK(hipDeviceSynchronize());
  const size_t G = num_cus();
  struct V {
    std::string name;
    std::function<void(float *, const float *)> f;
  };
  std::vector<V> vs = {
      {"prod ZIN (RT20)", [](float *y, const float *x) {
         BucketPtrs b = {};
         b.p[0] = x;
         launch_bucket_sum_nb<1, true>(y, nullptr, b, kN, 0);
       }},
      {"ZIN RT0 (2 chunks/launch)", [](float *y, const float *x) { fixed_chunks<0, true>(y, x); }},
      {"ZIN RT4", [](float *y, const float *x) { fixed_chunks<4, true>(y, x); }},
      {"ZIN RT12", [](float *y, const float *x) { fixed_chunks<12, true>(y, x); }},
      {"ZIN RT28", [](float *y, const float *x) { fixed_chunks<28, true>(y, x); }},
      {"stream /2", [=](float *y, const float *x) {
         hipLaunchKernelGGL(zin_stream, dim3(G * 2), dim3(kBlock), 0, 0, reinterpret_cast<f4 *>(y),
                            reinterpret_cast<const f4 *>(x), kN / 4);
       }},
      {"stream /4", [=](float *y, const float *x) {
         hipLaunchKernelGGL(zin_stream, dim3(G * 4), dim3(kBlock), 0, 0, reinterpret_cast<f4 *>(y),
                            reinterpret_cast<const f4 *>(x), kN / 4);
       }},
      {"add 1 bucket (prod)", [](float *y, const float *x) {
         BucketPtrs b = {};
         b.p[0] = x;
         launch_bucket_sum_nb<1>(y, y, b, kN, 0);
       }},
      {"memcpy D2D", [](float *y, const float *x) { CK(hipMemcpyAsync(y, x, kN * 4, hipMemcpyDeviceToDevice, 0)); }},
  };
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  std::vector<std::vector<std::vector<float>>> ms(bufs.size(), std::vector<std::vector<float>>(vs.size()));
  for (auto &bf : bufs)
    for (auto &v : vs) v.f(bf.y, bf.x);
  CK(hipDeviceSynchronize());
  for (int r = 0; r < rounds; ++r)
    for (size_t k = 0; k < bufs.size(); ++k)
      for (size_t i = 0; i < vs.size(); ++i) {
        CK(hipEventRecord(a, 0));
        vs[i].f(bufs[k].y, bufs[k].x);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float t = 0;
        CK(hipEventElapsedTime(&t, a, b));
        ms[k][i].push_back(t);
      }
  CK(hipGetLastError());
  for (size_t k = 0; k < bufs.size(); ++k)
    for (size_t i = 0; i < vs.size(); ++i) {
      auto m = ms[k][i];
      std::sort(m.begin(), m.end());
      const double med = m[m.size() / 2];
      const double bytes = (vs[i].name.rfind("add", 0) == 0 ? 3.0 : 2.0) * kN * 4;
      std::printf("alloc %zu %-28s %8.4f ms %6.1f%%\n", k, vs[i].name.c_str(), med,
                  100.0 * bytes / (med * 1e-3) / 8e12);
    }
  return 0;
}
