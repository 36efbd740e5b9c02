// persist_tune.hip — one launch per chunk vs a persistent launch with in-kernel
// phase alignment, for the phase-separated bucket sums (tuning harness, not
// product code; it #includes the product kernels).
//
// Production issues one launch per chunk: the launch boundary realigns the
// 256 blocks (one per CU) so that the chip reads, then writes, then reads the
// next chunk.  Against the same box's read-only / write-only stream rates each
// launch runs ~5 us over its no-mixing model: ~5 % of an 8-way sweep launch,
// ~8 % of a 2-bucket launch and ~12 % of a zero-input (copy) launch.  Here the
// chunks run in one persistent launch instead, and blocks align on a global
// arrival counter (vector atomics, relaxed; no data moves between blocks, so
// the counter only shapes timing and can never change a result).  Every wait
// is bounded (kMaxPolls sleeps), so the launch drains even if some block were
// not resident.
//   mode 0  launch per chunk (the production schedule, this file's kernel)
//   mode 1  persistent, no alignment
//   mode 2  persistent, align before each write phase
//   mode 3  persistent, align before each read phase
//   mode 4  persistent, both
// Forms: the 8-bucket sweep (RT 6, TG 4), the 2-bucket tile-major phased form
// (RT 20) and the zero-input 1-bucket form (RT 20: the planned init's dense
// runs).  Every result is compared bit for bit with production's.  Modes 2
// and 4 are run for the zero-input form only: with its register tiles live
// across the wait, the 8- and 2-bucket forms spilled to scratch (2 KiB/lane).
// Usage: persist_tune [rounds] [arenas]
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
constexpr unsigned kMaxPolls = 4096;        // x s_sleep(2) ~ 0.5 ms at most per wait

__device__ __forceinline__ void align_blocks(unsigned *ctr, unsigned target) {
  __syncthreads();
  // wave 0 arrives and polls; the poll loop is wave-uniform (readfirstlane),
  // so the register tiles live across it without divergent-loop handling
  const unsigned wave = __builtin_amdgcn_readfirstlane(threadIdx.x) >> 6;
  if (wave == 0) {
    if (threadIdx.x == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (unsigned n = 0; n < kMaxPolls; ++n) {
      const unsigned seen = __builtin_amdgcn_readfirstlane(
          __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      if (seen >= target) break;
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
}

// FORM 0: sweep (stream by stream), FORM 1: tile-major.  Chunks [c0, c1).
template <int FORM, int NB, int RT, bool ZIN, int MODE>
__global__ __launch_bounds__(kBlock) void persist_k(f4 *__restrict__ out, const f4 *__restrict__ in,
                                                    BucketPtrs b, size_t c0, size_t c1,
                                                    unsigned *ctr) {
  constexpr int U = kPhaseU;
  constexpr int TG = kSweepTG;
  constexpr int kT = kPhaseLdsTiles + RT;
  static_assert(FORM == 1 || kT % TG == 0, "whole bursts");
  __shared__ f4 res[kPhaseLdsF4];
  f4 keep[RT][U];
  const f4 *src[NB + 1];
  src[0] = in;
#pragma unroll
  for (int k = 0; k < NB; ++k) src[k + 1] = reinterpret_cast<const f4 *>(b.p[k]);
  const size_t G = gridDim.x;
  unsigned phase = 0;
  for (size_t c = c0; c < c1; ++c) {
    const size_t lo = c * G * (size_t)kT * kPhaseTile;
    if ((MODE == 3 || MODE == 4) && c > c0) align_blocks(ctr, (++phase) * (unsigned)G);
    if (FORM == 0) {
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
    } else {
#pragma unroll
      for (int t = 0; t < kT; ++t) {
        const size_t base = lo + ((size_t)t * G + blockIdx.x) * kPhaseTile + threadIdx.x;
        f4 acc[U];
        f4 v[NB][U];
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] = ZIN ? f4(0.0f) : ld_stream(in + base + u * kBlock);
#pragma unroll
        for (int k = 0; k < NB; ++k)
#pragma unroll
          for (int u = 0; u < U; ++u) v[k][u] = ld_stream(src[k + 1] + base + u * kBlock);
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
          for (int k = 0; k < NB; ++k) acc[u] += v[k][u];
          if (t < kPhaseLdsTiles)
            res[t * kPhaseTile + u * kBlock + threadIdx.x] = acc[u];
          else
            keep[t >= kPhaseLdsTiles ? t - kPhaseLdsTiles : 0][u] = acc[u];
        }
      }
    }
    if (MODE == 2 || MODE == 4)
      align_blocks(ctr + 1, (unsigned)(c - c0 + 1) * (unsigned)G);
    else
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
    __syncthreads();  // LDS slots are reused by the next chunk's read phase
  }
}

unsigned *g_ctr = nullptr;

// whole chunks of a 4 GiB shard; returns the floats covered
template <int FORM, int NB, int RT, bool ZIN, int MODE>
size_t run_k(float *out, const float *in, const BucketPtrs &b, bool run) {
  const size_t G = (size_t)num_cus();
  const size_t chunk_f4 = G * (size_t)(kPhaseLdsTiles + RT) * kPhaseTile;
  const size_t chunks = kN / 4 / chunk_f4;
  if (run) {
    if (MODE == 0) {
      for (size_t c = 0; c < chunks; ++c)
        hipLaunchKernelGGL((persist_k<FORM, NB, RT, ZIN, 0>), dim3((unsigned)G), dim3(kBlock), 0, 0,
                           reinterpret_cast<f4 *>(out), reinterpret_cast<const f4 *>(in), b, c, c + 1,
                           g_ctr);
    } else {
      CK(hipMemsetAsync(g_ctr, 0, 64, 0));
      hipLaunchKernelGGL((persist_k<FORM, NB, RT, ZIN, MODE>), dim3((unsigned)G), dim3(kBlock), 0, 0,
                         reinterpret_cast<f4 *>(out), reinterpret_cast<const f4 *>(in), b, (size_t)0, chunks,
                         g_ctr);
    }
  }
  return chunks * chunk_f4 * 4;
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
  CK(hipMalloc(&g_ctr, 64));
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
  // kind: nb = buckets summed into the master in place; nb = 0: zero-input
  // form, bucket 0 -> master (out = 0.0f + b0), as the planned init's runs.
  struct V {
    std::string name;
    int nb;
    std::function<size_t(float *, const BucketPtrs &, bool)> run;
  };
  auto prod_sum = [](int nb) {
    return [nb](float *m, const BucketPtrs &b, bool run) {
      std::vector<const float *> bv(b.p, b.p + nb);
      if (run) gp_bucket_sum_apply(m, bv.data(), nb, kN, nullptr);
      return kN;
    };
  };
  auto prod_zin = [](float *m, const BucketPtrs &b, bool run) {
    if (run) launch_bucket_sum_nb<1, true>(m, nullptr, b, kN, nullptr);
    return kN;
  };
#define SW(MODE) [](float *m, const BucketPtrs &b, bool r) { return run_k<0, 8, kSweepRT, false, MODE>(m, m, b, r); }
#define T2(MODE) [](float *m, const BucketPtrs &b, bool r) { return run_k<1, 2, 20, false, MODE>(m, m, b, r); }
#define Z1(MODE) [](float *m, const BucketPtrs &b, bool r) { return run_k<1, 1, 20, true, MODE>(m, nullptr, b, r); }
  std::vector<V> kinds = {
      {"prod sweep", 8, prod_sum(8)},
      {"m0 launch/chunk", 8, SW(0)},
      {"m1 persistent", 8, SW(1)},
      {"m3 align before read", 8, SW(3)},
      {"prod phased", 2, prod_sum(2)},
      {"m0 launch/chunk", 2, T2(0)},
      {"m1 persistent", 2, T2(1)},
      {"m3 align before read", 2, T2(3)},
      {"prod zin", 0, prod_zin},
      {"m0 launch/chunk", 0, Z1(0)},
      {"m1 persistent", 0, Z1(1)},
      {"m2 align before write", 0, Z1(2)},
      {"m3 align before read", 0, Z1(3)},
      {"m4 align both", 0, Z1(4)},
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
      std::printf("NB%d %-24s vs prod, %zu covered floats: %llu mismatches\n", v.nb, v.name.c_str(), covered,
                  hb);
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
      const double streams = v.nb == 0 ? 2.0 : v.nb + 2.0;
      rs.push_back(R{s.name + " NB" + std::to_string(v.nb) + " " + v.name, [=]() { f(m, bp, true); },
                     streams * covered * 4, {}});
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
