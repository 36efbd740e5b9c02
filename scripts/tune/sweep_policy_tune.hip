// sweep_policy_tune.hip — cache policy of the sweep-form bucket sum's master
// stream (tuning harness, not product code; it #includes the product kernels).
// Production loads every stream and stores the master non-temporally; the
// write probe (probe_tune.hip) streamed plain stores faster than non-temporal
// ones (6.3 vs 5.8 TB/s), so this A/Bs the master's load (ML) and store (MS)
// policy: 0 = non-temporal, 1 = plain.  Bit-identical by construction; checked.
// Usage: sweep_policy_tune [rounds] [arenas]
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

template <int NB, int ML, int MS>
__global__ __launch_bounds__(kBlock) void sweep_var(f4 *__restrict__ out, const f4 *__restrict__ in,
                                                    BucketPtrs b, size_t n4_tiles, size_t chunk) {
  constexpr int U = kPhaseU, RT = kSweepRT, TG = kSweepTG;
  constexpr int kT = kPhaseLdsTiles + RT;
  __shared__ f4 res[kPhaseLdsF4];
  f4 keep[RT][U];
  const f4 *src[NB + 1];
  src[0] = in;
#pragma unroll
  for (int k = 0; k < NB; ++k) src[k + 1] = reinterpret_cast<const f4 *>(b.p[k]);
  const size_t G = gridDim.x;
  const size_t lo = chunk * G * (size_t)kT * kPhaseTile;
  if (lo >= n4_tiles) return;
#pragma unroll
  for (int k = 0; k <= NB; ++k) {
#pragma unroll
    for (int t0 = 0; t0 < kT; t0 += TG) {
      f4 v[TG][U];
#pragma unroll
      for (int j = 0; j < TG; ++j)
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const f4 *p = src[k] + lo + ((size_t)(t0 + j) * G + blockIdx.x) * kPhaseTile + threadIdx.x +
                        u * kBlock;
          v[j][u] = (k == 0 && ML == 1) ? *p : ld_stream(p);
        }
#pragma unroll
      for (int j = 0; j < TG; ++j) {
        const int t = t0 + j;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (t < kPhaseLdsTiles) {
            f4 &r = res[t * kPhaseTile + u * kBlock + threadIdx.x];
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
    for (int u = 0; u < U; ++u) {
      const f4 v = t < kPhaseLdsTiles ? res[t * kPhaseTile + u * kBlock + threadIdx.x]
                                      : keep[t >= kPhaseLdsTiles ? t - kPhaseLdsTiles : 0][u];
      if (MS == 1)
        out[base + u * kBlock] = v;
      else
        __builtin_nontemporal_store(v, out + base + u * kBlock);
    }
  }
}

template <int NB, int ML, int MS>
void launch_var(float *m, const BucketPtrs &b) {
  const size_t n4 = kN / 4;
  const size_t G = (size_t)num_cus();
  const size_t chunk_f4 = G * (size_t)kSweepT * kPhaseTile;
  for (size_t c = 0; c < n4 / chunk_f4; ++c)
    hipLaunchKernelGGL((sweep_var<NB, ML, MS>), dim3((unsigned)G), dim3(kBlock), 0, 0,
                       reinterpret_cast<f4 *>(m), reinterpret_cast<const f4 *>(m), b, n4, c);
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

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 5;
  const int n_arenas = argc > 2 ? std::atoi(argv[2]) : 2;
  struct Set {
    std::string name;
    BucketPtrs b;
    float *master;
  };
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
  auto prod = [](int nb) {
    return [nb](float *m, const BucketPtrs &b) {
      std::vector<const float *> bv(b.p, b.p + nb);
      gp_bucket_sum_apply(m, bv.data(), nb, kN, nullptr);
    };
  };
  std::vector<V> kinds = {
      {"prod (ML nt, MS nt)", 8, prod(8)},
      {"ML nt, MS plain", 8, [](float *m, const BucketPtrs &b) { launch_var<8, 0, 1>(m, b); }},
      {"ML plain, MS nt", 8, [](float *m, const BucketPtrs &b) { launch_var<8, 1, 0>(m, b); }},
      {"ML plain, MS plain", 8, [](float *m, const BucketPtrs &b) { launch_var<8, 1, 1>(m, b); }},
      {"prod (ML nt, MS nt)", 4, prod(4)},
      {"ML nt, MS plain", 4, [](float *m, const BucketPtrs &b) { launch_var<4, 0, 1>(m, b); }},
      {"ML plain, MS plain", 4, [](float *m, const BucketPtrs &b) { launch_var<4, 1, 1>(m, b); }},
  };
  {
    const Set &s = sets[0];
    float *ref = nullptr, *m2 = nullptr;
    unsigned long long *bad = nullptr;
    CK(hipMalloc(&ref, kN * 4));
    CK(hipMalloc(&m2, kN * 4));
    CK(hipMalloc(&bad, 8));
    for (auto &v : kinds) {
      if (v.name.rfind("prod", 0) == 0) {
        CK(hipMemcpy(ref, s.master, kN * 4, hipMemcpyDeviceToDevice));
        v.run(ref, s.b);
        continue;
      }
      CK(hipMemcpy(m2, s.master, kN * 4, hipMemcpyDeviceToDevice));
      v.run(m2, s.b);
      CK(hipMemset(bad, 0, 8));
      diff_k<<<4096, 256>>>(reinterpret_cast<const unsigned *>(ref), reinterpret_cast<const unsigned *>(m2),
                            kN, bad);
      unsigned long long hb = 0;
      CK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
      std::printf("NB%d %-22s vs prod, all %zu floats: %llu mismatches\n", v.nb, v.name.c_str(), kN, hb);
    }
    CK(hipFree(ref));
    CK(hipFree(m2));
    CK(hipFree(bad));
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
  for (int k = 0; k < rounds; ++k)
    for (auto &r : rs) {
      CK(hipEventRecord(a));
      r.run();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      r.ms.push_back(ms);
    }
  std::printf("%-40s %10s %10s %10s %8s\n", "arena / kernel", "med_ms", "min_ms", "GB/s", "frac8T");
  for (auto &r : rs) {
    std::sort(r.ms.begin(), r.ms.end());
    const double med = r.ms[r.ms.size() / 2];
    const double gbs = r.bytes / (med * 1e-3) / 1e9;
    std::printf("%-40s %10.4f %10.4f %10.1f %8.4f\n", r.name.c_str(), med, r.ms[0], gbs, gbs / 8000.0);
  }
  return 0;
}
