// balance_tune.hip — balanced chunks for the phased bucket sum, and the phased
// form for shards below 3 chunks (tuning harness, not product code; it
// #includes the product kernels).
//
// Production splits a shard into fixed chunks of G x (10 + RT) tiles, so the
// last chunk can be tiny (the 512-MiB shard of an 8-GPU run at 8 buckets:
// 9.14 chunks -> a 10th launch of 2 tiles per block), and shards below 3
// chunks take the mixed form.  Here: C = ceil(tiles / (G x (10 + RT))) chunks
// of T = ceil(tiles / (G x C)) tiles per block each, down to a single chunk.
// Usage: balance_tune [rounds]
#include "../../geeps_amd/csrc/gp_reduce.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

template <int NB, int RT>
__global__ __launch_bounds__(kBlock) void bsum_bal(f4 *__restrict__ out, const f4 *__restrict__ in,
                                                   BucketPtrs b, size_t n4_tiles, size_t chunk,
                                                   int T) {
  constexpr int U = kPhaseU;
  constexpr int kT = kPhaseLdsTiles + RT;
  __shared__ f4 res[kPhaseLdsF4];
  f4 keep[RT > 0 ? RT : 1][U];
  const size_t G = gridDim.x;
  const size_t lo = chunk * G * (size_t)T * kPhaseTile;
#pragma unroll
  for (int t = 0; t < kT; ++t) {
    const size_t tile0 = lo + ((size_t)t * G + blockIdx.x) * kPhaseTile;
    if (t >= T || tile0 >= n4_tiles) break;
    const size_t base = tile0 + threadIdx.x;
    f4 acc[U], v[NB][U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = ld_stream(in + base + u * kBlock);
#pragma unroll
    for (int k = 0; k < NB; ++k)
#pragma unroll
      for (int u = 0; u < U; ++u) v[k][u] = ld_stream(reinterpret_cast<const f4 *>(b.p[k]) + base + u * kBlock);
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int k = 0; k < NB; ++k) acc[u] += v[k][u];
      if (t < kPhaseLdsTiles) res[t * kPhaseTile + u * kBlock + threadIdx.x] = acc[u];
      else keep[t >= kPhaseLdsTiles ? t - kPhaseLdsTiles : 0][u] = acc[u];
    }
  }
  __syncthreads();
#pragma unroll
  for (int t = 0; t < kT; ++t) {
    const size_t tile0 = lo + ((size_t)t * G + blockIdx.x) * kPhaseTile;
    if (t >= T || tile0 >= n4_tiles) break;
    const size_t base = tile0 + threadIdx.x;
#pragma unroll
    for (int u = 0; u < U; ++u)
      __builtin_nontemporal_store(t < kPhaseLdsTiles ? res[t * kPhaseTile + u * kBlock + threadIdx.x]
                                                     : keep[t >= kPhaseLdsTiles ? t - kPhaseLdsTiles : 0][u],
                                  out + base + u * kBlock);
  }
}

template <int NB, int RT>
void launch_bal(float *m, const BucketPtrs &b, size_t n) {
  const size_t n4_tiles = n / 4 / kPhaseTile * kPhaseTile;
  const size_t G = num_cus();
  const size_t tiles = n4_tiles / kPhaseTile;
  const size_t per = G * (kPhaseLdsTiles + RT);
  const size_t C = (tiles + per - 1) / per;
  const int T = (int)((tiles + G * C - 1) / (G * C));
  for (size_t c = 0; c < C; ++c)
    hipLaunchKernelGGL((bsum_bal<NB, RT>), dim3((unsigned)G), dim3(kBlock), 0, 0, reinterpret_cast<f4 *>(m),
                       reinterpret_cast<const f4 *>(m), b, n4_tiles, c, T);
  // the < 1-tile rest (none at the sizes below) would go to the mixed form
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
  const size_t kMaxN = (size_t)512 << 18;  // 512 MiB of floats per buffer
  char *a = nullptr;
  CK(hipMalloc(&a, 9 * kMaxN * 4));
  BucketPtrs bp = {};
  for (int k = 0; k < 8; ++k) {
    bp.p[k] = reinterpret_cast<const float *>(a + (size_t)k * kMaxN * 4);
    fill_k<<<4096, 256>>>(reinterpret_cast<float *>(a + (size_t)k * kMaxN * 4), kMaxN, 1000 + k);
  }
  float *m = reinterpret_cast<float *>(a + (size_t)8 * kMaxN * 4);
  fill_k<<<4096, 256>>>(m, kMaxN, 77);
  CK(hipDeviceSynchronize());
  std::vector<const float *> bv(bp.p, bp.p + 8);

  // correctness: balanced == production, bitwise, at every size and bucket count below
  const std::vector<size_t> sizes_mib = {8, 30, 64, 100, 200, 512};
  {
    float *m2 = nullptr;
    CK(hipMalloc(&m2, kMaxN * 4));
    size_t bad = 0;
    std::vector<float> h1(kMaxN), h2(kMaxN);
    for (size_t mib : sizes_mib) {
      const size_t n = mib << 18;
      CK(hipMemcpy(m2, m, n * 4, hipMemcpyDeviceToDevice));
      gp_bucket_sum_apply(m, bv.data(), 8, n, nullptr);
      launch_bal<8, 4>(m2, bp, n);
      gp_bucket_sum_apply(m, bv.data(), 1, n, nullptr);
      launch_bal<1, 20>(m2, bp, n);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(h1.data(), m, n * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(h2.data(), m2, n * 4, hipMemcpyDeviceToHost));
      bad += std::memcmp(h1.data(), h2.data(), n * 4) != 0;
    }
    std::printf("balanced vs production: %zu sizes mismatch\n", bad);
    CK(hipFree(m2));
  }

  struct V {
    std::string name;
    double bytes;
    std::function<void()> run;
    std::vector<float> ms;
  };
  std::vector<V> vs;
  for (size_t mib : sizes_mib) {
    const size_t n = mib << 18;
    for (int nb : {1, 8}) {
      const double bytes = (nb + 2.0) * n * 4;
      const std::string tag = std::to_string(mib) + " MiB NB" + std::to_string(nb);
      vs.push_back(V{tag + " prod", bytes, [=]() { gp_bucket_sum_apply(m, bv.data(), nb, n, nullptr); }, {}});
      if (nb == 8) {
        vs.push_back(V{tag + " bal RT4", bytes, [=]() { launch_bal<8, 4>(m, bp, n); }, {}});
        vs.push_back(V{tag + " bal RT0", bytes, [=]() { launch_bal<8, 0>(m, bp, n); }, {}});
      } else {
        vs.push_back(V{tag + " bal RT20", bytes, [=]() { launch_bal<1, 20>(m, bp, n); }, {}});
        vs.push_back(V{tag + " bal RT0", bytes, [=]() { launch_bal<1, 0>(m, bp, n); }, {}});
      }
    }
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto &v : vs) v.run();
  CK(hipDeviceSynchronize());
  for (int r = 0; r < rounds; ++r)
    for (auto &v : vs) {
      CK(hipEventRecord(e0));
      v.run();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.ms.push_back(ms);
    }
  std::printf("%-26s %10s %10s %10s %8s\n", "size / kernel", "med_ms", "min_ms", "GB/s", "frac8T");
  for (auto &v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const double med = v.ms[v.ms.size() / 2];
    const double gbs = v.bytes / (med * 1e-3) / 1e9;
    std::printf("%-26s %10.4f %10.4f %10.1f %8.4f\n", v.name.c_str(), med, v.ms[0], gbs, gbs / 8000.0);
  }
  return 0;
}
