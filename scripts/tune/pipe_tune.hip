// pipe_tune.hip — does software-pipelining the phased sum's read phase pay?
// (tuning harness, not product code; it #includes the product kernels)
//
// The production bucket_sum_phased_kernel issues a tile's (NB+1)*4 loads, waits
// for all of them (vmcnt(0)), sums them into LDS/registers, and only then issues
// the next tile's loads: with one wave per SIMD, each CU's load queue drains to
// empty at every tile boundary (14 per chunk at 8 buckets).  Here the read
// phase is split into stages of UH block-strides; stage s+1's loads are issued
// before stage s is consumed, so between (NB+1)*UH and 2*(NB+1)*UH loads stay
// in flight.  UH = 2 keeps production's register footprint (2 x 18 f4 at 8
// buckets); UH = 4 doubles it.  Same chunking, same tiles, same add order:
// bit-identical to production.  Usage: pipe_tune [rounds] [arenas]
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

template <int NB, int RT, int UH>
__global__ __launch_bounds__(kBlock) void bsum_pipe(f4 *__restrict__ out, const f4 *__restrict__ in,
                                                    BucketPtrs b, size_t n4_tiles, size_t chunk0) {
  constexpr int U = kPhaseU;
  constexpr int kT = kPhaseLdsTiles + RT;
  constexpr int SPT = U / UH;  // stages per tile
  constexpr int NS = kT * SPT;
  __shared__ f4 res[kPhaseLdsF4];
  f4 keep[RT > 0 ? RT : 1][U];
  const f4 *src[NB + 1];
  src[0] = in;
#pragma unroll
  for (int k = 0; k < NB; ++k) src[k + 1] = reinterpret_cast<const f4 *>(b.p[k]);
  const size_t G = gridDim.x;
  const size_t lo = chunk0 * G * (size_t)kT * kPhaseTile;
  if (lo >= n4_tiles) return;
  // tiles of this block in this chunk: t < nt (block-uniform)
  // Only whole chunks come here (every block has all kT tiles): the guards
  // below fold away, which keeps the waitcnt counts exact across stages.
  constexpr int nt = kT;
  constexpr int ns = NS;
  f4 buf[2][NB + 1][UH];
#define STAGE_BASE(s) \
  (lo + ((size_t)((s) / SPT) * G + blockIdx.x) * kPhaseTile + threadIdx.x + ((s) % SPT) * UH * kBlock)
  if (ns > 0) {
#pragma unroll
    for (int k = 0; k <= NB; ++k)
#pragma unroll
      for (int u = 0; u < UH; ++u) buf[0][k][u] = ld_stream(src[k] + STAGE_BASE(0) + u * kBlock);
  }
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    // fixed trip count, block-uniform guards (a break here kept the loop rolled)
    if (s + 1 < ns) {
#pragma unroll
      for (int k = 0; k <= NB; ++k)
#pragma unroll
        for (int u = 0; u < UH; ++u)
          buf[(s + 1) & 1][k][u] = ld_stream(src[k] + STAGE_BASE(s + 1) + u * kBlock);
    }
    const int t = s / SPT;
    if (s < ns) {
#pragma unroll
    for (int u = 0; u < UH; ++u) {
      f4 acc = buf[s & 1][0][u];
#pragma unroll
      for (int k = 1; k <= NB; ++k) acc += buf[s & 1][k][u];  // bucket order 0..NB-1
      const int uu = (s % SPT) * UH + u;
      if (t < kPhaseLdsTiles)
        res[t * kPhaseTile + uu * kBlock + threadIdx.x] = acc;
      else
        keep[t >= kPhaseLdsTiles ? t - kPhaseLdsTiles : 0][uu] = acc;
    }
    }
  }
#undef STAGE_BASE
  __syncthreads();
#pragma unroll
  for (int t = 0; t < kT; ++t) {
    if (t >= nt) continue;
    const size_t base = lo + ((size_t)t * G + blockIdx.x) * kPhaseTile + threadIdx.x;
#pragma unroll
    for (int u = 0; u < U; ++u)
      __builtin_nontemporal_store(t < kPhaseLdsTiles ? res[t * kPhaseTile + u * kBlock + threadIdx.x]
                                                     : keep[t >= kPhaseLdsTiles ? t - kPhaseLdsTiles : 0][u],
                                  out + base + u * kBlock);
  }
}

// Whole tiles of a 4 GiB buffer (kN is a multiple of the tile), one chunk per launch.
template <int NB, int RT, int UH>
void launch_pipe(float *m, const BucketPtrs &b) {
  const size_t n4 = kN / 4;
  const size_t G = (size_t)num_cus();
  const size_t chunk_f4 = G * (size_t)(kPhaseLdsTiles + RT) * kPhaseTile;
  const size_t full = n4 / chunk_f4;
  for (size_t c = 0; c < full; ++c)
    hipLaunchKernelGGL((bsum_pipe<NB, RT, UH>), dim3((unsigned)G), dim3(kBlock), 0, 0,
                       reinterpret_cast<f4 *>(m), reinterpret_cast<const f4 *>(m), b, n4, c);
  if (full * chunk_f4 < n4)  // the partial last chunk: production's kernel, same chunk geometry
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
      {"pipe RT4 UH2", 8, [](float *m, const BucketPtrs &b) { launch_pipe<8, 4, 2>(m, b); }},
      {"pipe RT4 UH4", 8, [](float *m, const BucketPtrs &b) { launch_pipe<8, 4, 4>(m, b); }},
      {"pipe RT8 UH2", 8, [](float *m, const BucketPtrs &b) { launch_pipe<8, 8, 2>(m, b); }},
      {"prod", 2, [](float *m, const BucketPtrs &b) {
         std::vector<const float *> bv(b.p, b.p + 2);
         gp_bucket_sum_apply(m, bv.data(), 2, kN, nullptr);
       }},
      {"pipe RT20 UH2", 2, [](float *m, const BucketPtrs &b) { launch_pipe<2, 20, 2>(m, b); }},
      {"pipe RT20 UH4", 2, [](float *m, const BucketPtrs &b) { launch_pipe<2, 20, 4>(m, b); }},
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
