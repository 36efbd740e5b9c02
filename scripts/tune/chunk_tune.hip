// chunk_tune.hip — chunk size of the sweep-form bucket sum (tuning harness,
// not product code; it #includes the product kernels)
//
// Production sums a 4 GiB shard at 3-8 buckets in 64 launches of one 64-MiB
// chunk each (16 tiles per block: 10 in LDS, 6 in registers).  Against the
// same box's read-only and write-only stream rates each launch is ~5 us over
// its no-mixing model (~95 us), i.e. what the launch boundary and the phase
// switch cost.  Bigger chunks (more register tiles, one wave per SIMD owns
// the whole register file) halve the launches.  This times the production
// kernel template at other RT / TG over whole chunks of a 4 GiB shard (bytes
// priced on the covered part only) and checks every covered float against
// production's result.
// Usage: chunk_tune [rounds] [arenas]
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

// whole chunks of the sweep kernel at RT / TG; returns the floats covered
template <int NB, int RT, int TG>
size_t launch_sweep(float *m, const BucketPtrs &b, bool run = true) {
  const size_t n4 = kN / 4;
  const size_t G = (size_t)num_cus();
  const size_t chunk_f4 = G * (size_t)(kPhaseLdsTiles + RT) * kPhaseTile;
  const size_t chunks = n4 / chunk_f4;
  if (run)
    for (size_t c = 0; c < chunks; ++c)
      hipLaunchKernelGGL((bucket_sum_sweep_kernel<NB, RT, TG>), dim3((unsigned)G), dim3(kBlock), 0, 0,
                         reinterpret_cast<f4 *>(m), reinterpret_cast<const f4 *>(m), b, n4, c);
  return chunks * chunk_f4 * 4;
}

template <int NB, int RT, int TG>
void report_attrs(const char *name) {
  hipFuncAttributes a;
  CK(hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&bucket_sum_sweep_kernel<NB, RT, TG>)));
  std::printf("%-26s regs %d  scratch %zu B/lane  lds %zu B\n", name, a.numRegs, a.localSizeBytes,
              a.sharedSizeBytes);
}


// The same sweep with buffer loads/stores: one resource per stream and
// chunk, the per-lane offset in one VGPR (threadIdx * 16) and the tile
// offset in an SGPR, so no 64-bit address pairs are held per load and the
// register tiles get the register file.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, bytes, 0x00020000);
}
typedef unsigned u4 __attribute__((ext_vector_type(4)));
constexpr int kAuxNT = 2;  // gfx94x/950 cache-policy bit 1: non-temporal

template <int NB, int RT, int TG>
__global__ __launch_bounds__(kBlock) void sweep_buf(f4 *__restrict__ out, const f4 *__restrict__ in,
                                                    BucketPtrs b, size_t n4_tiles, size_t chunk) {
  constexpr int U = kPhaseU;
  constexpr int kT = kPhaseLdsTiles + RT;
  static_assert(kT % TG == 0, "whole bursts");
  __shared__ f4 res[kPhaseLdsF4];
  f4 keep[RT][U];
  const size_t G = gridDim.x;
  const size_t lo = chunk * G * (size_t)kT * kPhaseTile;
  const uint32_t chunk_bytes = (uint32_t)(G * kT * kPhaseTile * 16);
  if (lo >= n4_tiles) return;
  const uint32_t voff = threadIdx.x * 16;
#pragma unroll
  for (int k = 0; k <= NB; ++k) {
    const f4 *s = k == 0 ? in : reinterpret_cast<const f4 *>(b.p[k > 0 ? k - 1 : 0]);
    const __amdgpu_buffer_rsrc_t r = rsrc(s + lo, chunk_bytes);
#pragma unroll
    for (int t0 = 0; t0 < kT; t0 += TG) {
      f4 v[TG][U];
#pragma unroll
      for (int j = 0; j < TG; ++j)
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint32_t soff = (uint32_t)(((t0 + j) * G + blockIdx.x) * kPhaseTile * 16) + u * kBlock * 16;
          v[j][u] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, kAuxNT));
        }
#pragma unroll
      for (int j = 0; j < TG; ++j) {
        const int t = t0 + j;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (t < kPhaseLdsTiles) {
            f4 &q = res[t * kPhaseTile + u * kBlock + threadIdx.x];
            q = k == 0 ? v[j][u] : q + v[j][u];
          } else {
            f4 &q = keep[t >= kPhaseLdsTiles ? t - kPhaseLdsTiles : 0][u];
            q = k == 0 ? v[j][u] : q + v[j][u];
          }
        }
      }
    }
  }
  __syncthreads();
  const __amdgpu_buffer_rsrc_t ro = rsrc(out + lo, chunk_bytes);
#pragma unroll
  for (int t = 0; t < kT; ++t) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t soff = (uint32_t)((t * G + blockIdx.x) * kPhaseTile * 16) + u * kBlock * 16;
      const f4 q = t < kPhaseLdsTiles ? res[t * kPhaseTile + u * kBlock + threadIdx.x]
                                      : keep[t >= kPhaseLdsTiles ? t - kPhaseLdsTiles : 0][u];
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, q), ro, voff, soff, kAuxNT);
    }
  }
}

template <int NB, int RT, int TG>
size_t launch_buf(float *m, const BucketPtrs &b, bool run = true) {
  const size_t n4 = kN / 4;
  const size_t G = (size_t)num_cus();
  const size_t chunk_f4 = G * (size_t)(kPhaseLdsTiles + RT) * kPhaseTile;
  const size_t chunks = n4 / chunk_f4;
  if (run)
    for (size_t c = 0; c < chunks; ++c)
      hipLaunchKernelGGL((sweep_buf<NB, RT, TG>), dim3((unsigned)G), dim3(kBlock), 0, 0,
                         reinterpret_cast<f4 *>(m), reinterpret_cast<const f4 *>(m), b, n4, c);
  return chunks * chunk_f4 * 4;
}

template <int NB, int RT, int TG>
void report_buf(const char *name) {
  hipFuncAttributes a;
  CK(hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&sweep_buf<NB, RT, TG>)));
  std::printf("%-26s regs %d  scratch %zu B/lane  lds %zu B\n", name, a.numRegs, a.localSizeBytes,
              a.sharedSizeBytes);
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
  report_attrs<8, 6, 4>("NB8 RT6 TG4 (prod)");
  report_attrs<8, 14, 4>("NB8 RT14 TG4");
  report_buf<8, 6, 4>("buf NB8 RT6 TG4");
  report_buf<8, 14, 4>("buf NB8 RT14 TG4");
  report_buf<8, 22, 4>("buf NB8 RT22 TG4");
  report_buf<8, 22, 2>("buf NB8 RT22 TG2");
  report_buf<4, 22, 4>("buf NB4 RT22 TG4");
  report_buf<3, 22, 4>("buf NB3 RT22 TG4");
  report_buf<2, 22, 4>("buf NB2 RT22 TG4");
  struct V {
    std::string name;
    int nb;
    std::function<size_t(float *, const BucketPtrs &, bool)> run;
  };
  auto prod = [](int nb) {
    return [nb](float *m, const BucketPtrs &b, bool run) {
      std::vector<const float *> bv(b.p, b.p + nb);
      if (run) gp_bucket_sum_apply(m, bv.data(), nb, kN, nullptr);
      return kN;
    };
  };
  std::vector<V> kinds = {
      {"prod (RT6 TG4, 64 MiB)", 8, prod(8)},
      {"RT14 TG4 (96 MiB)", 8, [](float *m, const BucketPtrs &b, bool r) { return launch_sweep<8, 14, 4>(m, b, r); }},
      {"buf RT6 TG4 (64 MiB)", 8, [](float *m, const BucketPtrs &b, bool r) { return launch_buf<8, 6, 4>(m, b, r); }},
      {"buf RT14 TG4 (96 MiB)", 8, [](float *m, const BucketPtrs &b, bool r) { return launch_buf<8, 14, 4>(m, b, r); }},
      {"buf RT22 TG4 (128 MiB)", 8, [](float *m, const BucketPtrs &b, bool r) { return launch_buf<8, 22, 4>(m, b, r); }},
      {"buf RT22 TG2 (128 MiB)", 8, [](float *m, const BucketPtrs &b, bool r) { return launch_buf<8, 22, 2>(m, b, r); }},
      {"prod (RT6 TG4, 64 MiB)", 4, prod(4)},
      {"buf RT22 TG4 (128 MiB)", 4, [](float *m, const BucketPtrs &b, bool r) { return launch_buf<4, 22, 4>(m, b, r); }},
      {"prod (RT6 TG4, 64 MiB)", 3, prod(3)},
      {"buf RT22 TG4 (128 MiB)", 3, [](float *m, const BucketPtrs &b, bool r) { return launch_buf<3, 22, 4>(m, b, r); }},
      {"prod (phased RT20)", 2, prod(2)},
      {"buf sweep RT22 TG4 (128 MiB)", 2, [](float *m, const BucketPtrs &b, bool r) { return launch_buf<2, 22, 4>(m, b, r); }},
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
        v.run(ref, s.b, true);
        continue;
      }
      CK(hipMemcpy(m2, s.master, kN * 4, hipMemcpyDeviceToDevice));
      const size_t covered = v.run(m2, s.b, true);
      CK(hipMemset(bad, 0, 8));
      diff_k<<<4096, 256>>>(reinterpret_cast<const unsigned *>(ref), reinterpret_cast<const unsigned *>(m2),
                            covered, bad);
      unsigned long long hb = 0;
      CK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
      std::printf("NB%d %-26s vs prod, %zu covered floats: %llu mismatches\n", v.nb, v.name.c_str(),
                  covered, hb);
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
      const size_t covered = f(m, bp, false);
      rs.push_back(R{s.name + " NB" + std::to_string(v.nb) + " " + v.name, [=]() { f(m, bp, true); },
                     (v.nb + 2.0) * covered * 4, {}});
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
  std::printf("%-46s %10s %10s %10s %8s\n", "arena / kernel", "med_ms", "min_ms", "GB/s", "frac8T");
  for (auto &r : rs) {
    std::sort(r.ms.begin(), r.ms.end());
    const double med = r.ms[r.ms.size() / 2];
    const double gbs = r.bytes / (med * 1e-3) / 1e9;
    std::printf("%-46s %10.4f %10.4f %10.1f %8.4f\n", r.name.c_str(), med, r.ms[0], gbs, gbs / 8000.0);
  }
  return 0;
}
