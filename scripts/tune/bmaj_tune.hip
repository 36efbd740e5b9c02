// bmaj_tune.hip — bucket-major read phase for the phased sum (tuning harness,
// not product code; it #includes the product kernels)
//
// Production's read phase walks a chunk tile by tile and loads all NB+1 streams
// of a tile together, so at any moment the chip reads 9 regions (master + 8
// buckets).  Here it walks the chunk once per stream instead, in bucket order:
// pass 0 loads the master's tiles into LDS/registers, pass k adds bucket k-1's
// tiles into them.  At any moment the chip then reads ONE contiguous region of
// one stream.  The per-element add order is unchanged (((m + b0) + b1) + ...),
// so the result is bit-identical.  TG tiles' loads are issued per burst.
// "prod" is whatever gp_reduce.hip ships (since the sweep form was adopted:
// the sweep kernel); "tile-major" is the plan before it.
// Usage: bmaj_tune [rounds] [arenas]
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

template <int NB, int RT, int TG>
__global__ __launch_bounds__(kBlock) void bsum_bmaj(f4 *__restrict__ out, const f4 *__restrict__ in,
                                                    BucketPtrs b, size_t n4_tiles, size_t chunk0) {
  constexpr int U = kPhaseU;
  constexpr int kT = kPhaseLdsTiles + RT;
  static_assert(kT % TG == 0, "bursts of TG tiles");
  __shared__ f4 res[kPhaseLdsF4];
  f4 keep[RT > 0 ? RT : 1][U];
  const f4 *src[NB + 1];
  src[0] = in;
#pragma unroll
  for (int k = 0; k < NB; ++k) src[k + 1] = reinterpret_cast<const f4 *>(b.p[k]);
  const size_t G = gridDim.x;
  const size_t lo = chunk0 * G * (size_t)kT * kPhaseTile;  // whole chunks only
  if (lo >= n4_tiles) return;
#pragma unroll
  for (int k = 0; k <= NB; ++k) {
#pragma unroll
    for (int t0 = 0; t0 < kT; t0 += TG) {
      f4 v[TG][U];
#pragma unroll
      for (int j = 0; j < TG; ++j)
#pragma unroll
        for (int u = 0; u < U; ++u)
          v[j][u] = ld_stream(src[k] + lo + ((size_t)(t0 + j) * G + blockIdx.x) * kPhaseTile +
                              threadIdx.x + u * kBlock);
#pragma unroll
      for (int j = 0; j < TG; ++j) {
        const int t = t0 + j;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (t < kPhaseLdsTiles) {
            f4 &r = res[t * kPhaseTile + u * kBlock + threadIdx.x];  // own slot: no barrier
            r = k == 0 ? v[j][u] : r + v[j][u];
          } else {
            f4 &r = keep[t >= kPhaseLdsTiles ? t - kPhaseLdsTiles : 0][u];
            r = k == 0 ? v[j][u] : r + v[j][u];
          }
        }
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int t = 0; t < kT; ++t) {
    const size_t base = lo + ((size_t)t * G + blockIdx.x) * kPhaseTile + threadIdx.x;
#pragma unroll
    for (int u = 0; u < U; ++u)
      __builtin_nontemporal_store(t < kPhaseLdsTiles ? res[t * kPhaseTile + u * kBlock + threadIdx.x]
                                                     : keep[t >= kPhaseLdsTiles ? t - kPhaseLdsTiles : 0][u],
                                  out + base + u * kBlock);
  }
}

// Whole tiles of a 4 GiB buffer, one chunk per launch; the partial last chunk
// runs production's kernel with the same chunk geometry.
template <int NB, int RT, int TG>
void launch_bmaj(float *m, const BucketPtrs &b) {
  const size_t n4 = kN / 4;
  const size_t G = (size_t)num_cus();
  const size_t chunk_f4 = G * (size_t)(kPhaseLdsTiles + RT) * kPhaseTile;
  const size_t full = n4 / chunk_f4;
  for (size_t c = 0; c < full; ++c)
    hipLaunchKernelGGL((bsum_bmaj<NB, RT, TG>), dim3((unsigned)G), dim3(kBlock), 0, 0,
                       reinterpret_cast<f4 *>(m), reinterpret_cast<const f4 *>(m), b, n4, c);
  if (full * chunk_f4 < n4)
    hipLaunchKernelGGL((bucket_sum_phased_kernel<NB, RT, false>), dim3((unsigned)G), dim3(kBlock), 0, 0,
                       reinterpret_cast<f4 *>(m), reinterpret_cast<const f4 *>(m), b, n4, full, 0);
}

// The tile-major plan production used before the sweep form (whole tiles of a
// 4 GiB buffer, fixed register-tile chunks, one per launch).
template <int NB>
void launch_tilemajor(float *m, const BucketPtrs &b) {
  const size_t n4_tiles = kN / 4 / kPhaseTile * kPhaseTile;
  const PhasePlan p = phase_plan<NB>(n4_tiles);
  launch_phased<NB, phase_reg_tiles<NB>(), false>(m, m, b, n4_tiles, p, 0);
}

// The production sweep kernel at other shapes (RT register tiles, TG-tile bursts).
template <int NB, int RT, int TG>
void launch_sweep(float *m, const BucketPtrs &b) {
  const size_t n4 = kN / 4;
  const size_t G = (size_t)num_cus();
  const size_t chunk_f4 = G * (size_t)(kPhaseLdsTiles + RT) * kPhaseTile;
  const size_t full = n4 / chunk_f4;
  for (size_t c = 0; c < full; ++c)
    hipLaunchKernelGGL((bucket_sum_sweep_kernel<NB, RT, TG>), dim3((unsigned)G), dim3(kBlock), 0, 0,
                       reinterpret_cast<f4 *>(m), reinterpret_cast<const f4 *>(m), b, n4, c);
  if (full * chunk_f4 < n4)
    hipLaunchKernelGGL((bucket_sum_phased_kernel<NB, RT, false>), dim3((unsigned)G), dim3(kBlock), 0, 0,
                       reinterpret_cast<f4 *>(m), reinterpret_cast<const f4 *>(m), b, n4, full, 0);
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

__global__ void diff_k(const unsigned *a, const unsigned *b, size_t n, unsigned long long *bad) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  unsigned long long c = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) c += a[i] != b[i];
  if (c) atomicAdd(bad, c);
}

struct Set {
  std::string name;
  BucketPtrs b;
  float *master;
};

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 5;
  const int n_arenas = argc > 2 ? std::atoi(argv[2]) : 3;
  std::vector<Set> sets;
  for (int i = 0; i < n_arenas; ++i) {
    char *a = nullptr;
    const size_t stride = kN * 4;
    CK(hipMalloc(&a, 9 * stride));
    Set s{"arena #" + std::to_string(i + 1), {}, nullptr};
    for (int k = 0; k < 8; ++k) {
      s.b.p[k] = reinterpret_cast<const float *>(a + (size_t)k * stride);
      fill_k<<<4096, 256>>>(reinterpret_cast<float *>(a + (size_t)k * stride), kN, 1000 + k);
    }
    s.master = reinterpret_cast<float *>(a + (size_t)8 * stride);
    fill_k<<<4096, 256>>>(s.master, kN, 77);
    sets.push_back(s);
  }
  CK(hipDeviceSynchronize());

  struct V {
    std::string name;
    int nb;
    std::function<void(float *, const BucketPtrs &)> run;
  };
  std::vector<V> kinds = {
      {"prod", 8, [](float *m, const BucketPtrs &b) {
         std::vector<const float *> bv(b.p, b.p + 8);
         gp_bucket_sum_apply(m, bv.data(), 8, kN, nullptr);
       }},
      {"tile-major", 8, [](float *m, const BucketPtrs &b) { launch_tilemajor<8>(m, b); }},
      {"sweep RT4 TG7", 8, [](float *m, const BucketPtrs &b) { launch_sweep<8, 4, 7>(m, b); }},
      {"sweep RT6 TG2", 8, [](float *m, const BucketPtrs &b) { launch_sweep<8, 6, 2>(m, b); }},
      {"sweep RT6 TG8", 8, [](float *m, const BucketPtrs &b) { launch_sweep<8, 6, 8>(m, b); }},
      {"sweep RT8 TG6", 8, [](float *m, const BucketPtrs &b) { launch_sweep<8, 8, 6>(m, b); }},
      {"prod", 6, [](float *m, const BucketPtrs &b) {
         std::vector<const float *> bv(b.p, b.p + 6);
         gp_bucket_sum_apply(m, bv.data(), 6, kN, nullptr);
       }},
      {"tile-major", 6, [](float *m, const BucketPtrs &b) { launch_tilemajor<6>(m, b); }},
      {"sweep RT4 TG7", 6, [](float *m, const BucketPtrs &b) { launch_sweep<6, 4, 7>(m, b); }},
      {"prod", 5, [](float *m, const BucketPtrs &b) {
         std::vector<const float *> bv(b.p, b.p + 5);
         gp_bucket_sum_apply(m, bv.data(), 5, kN, nullptr);
       }},
      {"sweep RT4 TG7", 5, [](float *m, const BucketPtrs &b) { launch_sweep<5, 4, 7>(m, b); }},
      {"prod", 3, [](float *m, const BucketPtrs &b) {
         std::vector<const float *> bv(b.p, b.p + 3);
         gp_bucket_sum_apply(m, bv.data(), 3, kN, nullptr);
       }},
      {"tile-major", 3, [](float *m, const BucketPtrs &b) { launch_tilemajor<3>(m, b); }},
      {"sweep RT4 TG7", 3, [](float *m, const BucketPtrs &b) { launch_sweep<3, 4, 7>(m, b); }},
  };

  // correctness: every variant against production on copies of one master, all floats
  {
    const Set &s = sets[0];
    float *ref = nullptr, *m2 = nullptr;
    unsigned long long *bad = nullptr;
    CK(hipMalloc(&ref, kN * 4));
    CK(hipMalloc(&m2, kN * 4));
    CK(hipMalloc(&bad, 8));
    for (auto &v : kinds) {
      if (v.name == "prod") {
        CK(hipMemcpy(ref, s.master, kN * 4, hipMemcpyDeviceToDevice));
        v.run(ref, s.b);
        continue;
      }
      CK(hipMemcpy(m2, s.master, kN * 4, hipMemcpyDeviceToDevice));
      v.run(m2, s.b);
      CK(hipMemset(bad, 0, 8));
      diff_k<<<4096, 256>>>(reinterpret_cast<const unsigned *>(ref), reinterpret_cast<const unsigned *>(m2), kN,
                            bad);
      unsigned long long hb = 0;
      CK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
      std::printf("NB%d %-16s vs prod, all %zu floats: %llu mismatches\n", v.nb, v.name.c_str(), kN, hb);
    }
    CK(hipFree(ref));
    CK(hipFree(m2));
    CK(hipFree(bad));
    std::fflush(stdout);
  }

  struct R {
    std::string name;
    std::function<void()> run;
    double bytes;
    std::vector<float> ms;
  };
  std::vector<R> rs;
  for (auto &s : sets)
    for (auto &v : kinds) {
      float *m = s.master;
      BucketPtrs bp = s.b;
      auto f = v.run;
      rs.push_back(R{s.name + " NB" + std::to_string(v.nb) + " " + v.name, [=]() { f(m, bp); },
                     (v.nb + 2.0) * kN * 4, {}});
    }
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (auto &r : rs) r.run();
  CK(hipDeviceSynchronize());
  for (int k = 0; k < rounds; ++k) {
    for (auto &r : rs) {
      CK(hipEventRecord(a));
      r.run();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      r.ms.push_back(ms);
    }
  }
  std::printf("%-34s %10s %10s %10s %8s\n", "arena / kernel", "med_ms", "min_ms", "GB/s", "frac8T");
  for (auto &r : rs) {
    std::sort(r.ms.begin(), r.ms.end());
    const double med = r.ms[r.ms.size() / 2];
    const double gbs = r.bytes / (med * 1e-3) / 1e9;
    std::printf("%-34s %10.4f %10.4f %10.1f %8.4f\n", r.name.c_str(), med, r.ms[0], gbs, gbs / 8000.0);
  }
  return 0;
}
