// phase_tune.hip — does separating the 8-way bucket sum's reads from its writes
// in time beat the mixed stream?  (tuning harness, not product code; it
// #includes the product kernels)
//
// alloc_tune.hip showed that on every allocation the nine read streams alone
// take ≈5.6–5.7 ms and the master's write stream alone ≈0.8 ms, while the
// mixed kernel takes 7.2–8.4 ms depending on the allocation.  Here a CHUNK of
// the shard is summed into LDS by every CU (read phase: master + 8 buckets),
// then written back (write phase).  No grid barrier: each launch covers
// K chunks, and the CUs stay roughly in phase because they all do the same
// work and a launch starts them together.  Usage: phase_tune [rounds] [arenas]
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

// One block per CU / BPC per CU; LDS_F4 f4 results per block per chunk.
// Chunk c covers f4 [c * G * LDS_F4, (c + 1) * G * LDS_F4); inside it, block g
// takes 16-KiB tiles g, g + G, ... (U = 4 strides of 256 threads).
template <int NB, int LDS_F4, int K, int BS = kBlock, int U = 4, int POL = 0>
__global__ __launch_bounds__(BS) void bsum_phased(f4 *__restrict__ master, BucketPtrs b,
                                                  size_t n4, size_t chunk0) {
  constexpr int kTile = BS * U;                  // f4 per tile
  constexpr int kTilesPerBlock = LDS_F4 / kTile;  // per chunk
  __shared__ f4 res[LDS_F4];
  const size_t G = gridDim.x;
  const size_t chunk_f4 = G * LDS_F4;
  for (int kc = 0; kc < K; ++kc) {
    const size_t lo = (chunk0 + kc) * chunk_f4;
    if (lo >= n4) return;  // grid-uniform
    // read phase
    for (int t = 0; t < kTilesPerBlock; ++t) {
      const size_t base = lo + ((size_t)t * G + blockIdx.x) * kTile + threadIdx.x;
      if (base + (U - 1) * BS >= n4) break;  // harness sizes are whole chunks
      f4 acc[U];
      f4 v[NB][U];
#pragma unroll
      for (int u = 0; u < U; ++u)
        acc[u] = (POL & 1) ? __builtin_nontemporal_load(master + base + u * BS) : master[base + u * BS];
#pragma unroll
      for (int k = 0; k < NB; ++k)
#pragma unroll
        for (int u = 0; u < U; ++u)
          v[k][u] = __builtin_nontemporal_load(reinterpret_cast<const f4 *>(b.p[k]) + base + u * BS);
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int k = 0; k < NB; ++k) acc[u] += v[k][u];
        res[t * kTile + u * BS + threadIdx.x] = acc[u];
      }
    }
    __syncthreads();
    // write phase
    for (int t = 0; t < kTilesPerBlock; ++t) {
      const size_t base = lo + ((size_t)t * G + blockIdx.x) * kTile + threadIdx.x;
      if (base + (U - 1) * BS >= n4) break;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (POL & 2)
          __builtin_nontemporal_store(res[t * kTile + u * BS + threadIdx.x], master + base + u * BS);
        else
          master[base + u * BS] = res[t * kTile + u * BS + threadIdx.x];
      }
    }
    __syncthreads();
  }
}

template <int NB, int LDS_F4, int K, int BS = kBlock, int U = 4, int POL = 0>
void launch_phased(float *m, const BucketPtrs &b, int bpc) {
  const size_t n4 = kN / 4;
  const size_t G = (size_t)num_cus() * bpc;
  const size_t chunk_f4 = G * LDS_F4;
  const size_t chunks = (n4 + chunk_f4 - 1) / chunk_f4;
  for (size_t c = 0; c < chunks; c += K)
    hipLaunchKernelGGL((bsum_phased<NB, LDS_F4, K, BS, U, POL>), dim3((unsigned)G), dim3(BS), 0, 0,
                       reinterpret_cast<f4 *>(m), b, n4, c);
}

// Register-extended chunks: besides LDS_F4 f4 of results in LDS, each lane
// keeps RT more tiles' results in VGPRs (1 wave per SIMD leaves ~300 VGPRs
// for them), so a chunk per CU is (LDS_F4 / kTile + RT) tiles and the read and
// write phases are that much longer.
template <int NB, int LDS_F4, int RT, int K, int U = 4>
__global__ __launch_bounds__(kBlock) void bsum_phased_reg(f4 *__restrict__ master, BucketPtrs b,
                                                         size_t n4, size_t chunk0) {
  constexpr int BS = kBlock;
  constexpr int kTile = BS * U;
  constexpr int kLT = LDS_F4 / kTile;
  constexpr int kT = kLT + RT;  // tiles per block per chunk
  __shared__ f4 res[LDS_F4];
  const size_t G = gridDim.x;
  const size_t chunk_f4 = G * (size_t)kT * kTile;
  f4 keep[RT > 0 ? RT : 1][U];
  for (int kc = 0; kc < K; ++kc) {
    const size_t lo = (chunk0 + kc) * chunk_f4;
    if (lo >= n4) return;  // grid-uniform
#pragma unroll
    for (int t = 0; t < kT; ++t) {
      const size_t base = lo + ((size_t)t * G + blockIdx.x) * kTile + threadIdx.x;
      const bool live = base + (U - 1) * BS < n4;
      f4 acc[U];
      f4 v[NB][U];
      if (live) {
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] = __builtin_nontemporal_load(master + base + u * BS);
#pragma unroll
        for (int k = 0; k < NB; ++k)
#pragma unroll
          for (int u = 0; u < U; ++u)
            v[k][u] = __builtin_nontemporal_load(reinterpret_cast<const f4 *>(b.p[k]) + base + u * BS);
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
          for (int k = 0; k < NB; ++k) acc[u] += v[k][u];
          if (t < kLT) res[t * kTile + u * BS + threadIdx.x] = acc[u];
          else keep[t >= kLT ? t - kLT : 0][u] = acc[u];
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < kT; ++t) {
      const size_t base = lo + ((size_t)t * G + blockIdx.x) * kTile + threadIdx.x;
      if (base + (U - 1) * BS >= n4) continue;
#pragma unroll
      for (int u = 0; u < U; ++u)
        __builtin_nontemporal_store(t < kLT ? res[t * kTile + u * BS + threadIdx.x] : keep[t >= kLT ? t - kLT : 0][u],
                                    master + base + u * BS);
    }
    __syncthreads();
  }
}

template <int NB, int LDS_F4, int RT, int K, int U = 4>
void launch_phased_reg(float *m, const BucketPtrs &b) {
  const size_t n4 = kN / 4;
  const size_t G = (size_t)num_cus();
  const size_t chunk_f4 = G * (size_t)(LDS_F4 / (kBlock * U) + RT) * kBlock * U;
  const size_t chunks = (n4 + chunk_f4 - 1) / chunk_f4;
  for (size_t c = 0; c < chunks; c += K)
    hipLaunchKernelGGL((bsum_phased_reg<NB, LDS_F4, RT, K, U>), dim3((unsigned)G), dim3(kBlock), 0, 0,
                       reinterpret_cast<f4 *>(m), b, n4, c);
}

// The production kernel's fixed-chunk launches alternated over two streams, so
// chunk l + 1 can start on CUs that chunk l's tail has freed (no dependency:
// chunks are disjoint).  Blocking streams: the null-stream events around a
// call still bracket all of it.
template <int NB>
void launch_prod_two_streams(float *m, const BucketPtrs &b, hipStream_t s0, hipStream_t s1) {
  const size_t n4_tiles = kN / 4 / kPhaseTile * kPhaseTile;
  const PhasePlan p = phase_plan<NB>(n4_tiles);
  for (size_t l = 0; l < p.launches; ++l)
    hipLaunchKernelGGL((bucket_sum_phased_kernel<NB, phase_reg_tiles<NB>(), false>),
                       dim3((unsigned)num_cus()), dim3(kBlock), 0, (l & 1) ? s1 : s0,
                       reinterpret_cast<f4 *>(m), reinterpret_cast<const f4 *>(m), b, n4_tiles, l, 0);
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

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 5;
  std::vector<Set> sets;
  const int n_arenas = argc > 2 ? std::atoi(argv[2]) : 3;
  // PHASE_TUNE_PADS=1: arena i puts kPads[i % 5] bytes between consecutive
  // buffers, so a CU's nine same-offset loads fall on different HBM channels.
  const bool pads = std::getenv("PHASE_TUNE_PADS") != nullptr;
  const size_t kPads[5] = {0, 4096, 16384, 69632, (1u << 20) + 4096};
  for (int i = 0; i < n_arenas; ++i) {
    char *a = nullptr;
    const size_t pad = pads ? kPads[i % 5] : 0;
    const size_t stride = kN * 4 + pad;
    CK(hipMalloc(&a, 9 * stride));
    Set s{"arena #" + std::to_string(i + 1) + (pads ? " pad " + std::to_string(pad) : ""), {}, nullptr};
    for (int k = 0; k < 8; ++k) {
      s.b.p[k] = reinterpret_cast<const float *>(a + (size_t)k * stride);
      fill_k<<<4096, 256>>>(reinterpret_cast<float *>(a + (size_t)k * stride), kN, 1000 + k);
    }
    s.master = reinterpret_cast<float *>(a + (size_t)8 * stride);
    fill_k<<<4096, 256>>>(s.master, kN, 77);
    sets.push_back(s);
  }
  CK(hipDeviceSynchronize());

  // correctness: phased == production on a copy of the master (bitwise)
  {
    const Set &s = sets[0];
    float *m2 = nullptr;
    CK(hipMalloc(&m2, kN * 4));
    CK(hipMemcpy(m2, s.master, kN * 4, hipMemcpyDeviceToDevice));
    std::vector<const float *> bv(s.b.p, s.b.p + 8);
    gp_bucket_sum_apply(s.master, bv.data(), 8, kN, nullptr);
    launch_phased<8, 4096, 4>(m2, s.b, 2);
    CK(hipDeviceSynchronize());
    std::vector<float> h1(1 << 20), h2(1 << 20);
    size_t bad = 0;
    for (size_t off = 0; off < kN; off += kN / 8) {
      CK(hipMemcpy(h1.data(), s.master + off, h1.size() * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(h2.data(), m2 + off, h2.size() * 4, hipMemcpyDeviceToHost));
      for (size_t i = 0; i < h1.size(); ++i) bad += std::memcmp(&h1[i], &h2[i], 4) != 0;
    }
    CK(hipMemcpy(h1.data(), s.master + kN - h1.size(), h1.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h2.data(), m2 + kN - h2.size(), h2.size() * 4, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < h1.size(); ++i) bad += std::memcmp(&h1[i], &h2[i], 4) != 0;
    std::printf("phased vs production, sampled 9 Mi floats: %zu mismatches\n", bad);
    // register-extended form: full compare against production on fresh copies
    CK(hipMemcpy(m2, s.master, kN * 4, hipMemcpyDeviceToDevice));
    gp_bucket_sum_apply(s.master, bv.data(), 8, kN, nullptr);
    launch_phased_reg<8, 10240, 12, 1>(m2, s.b);
    CK(hipDeviceSynchronize());
    size_t bad2 = 0;
    for (size_t off = 0; off < kN; off += h1.size()) {
      CK(hipMemcpy(h1.data(), s.master + off, h1.size() * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(h2.data(), m2 + off, h2.size() * 4, hipMemcpyDeviceToHost));
      bad2 += std::memcmp(h1.data(), h2.data(), h1.size() * 4) != 0;
    }
    std::printf("register-extended phased vs production, all floats: %zu mismatching 4-MiB blocks\n", bad2);
    CK(hipFree(m2));
  }

  struct V {
    std::string name;
    std::function<void()> run;
    std::vector<float> ms;
  };
  std::vector<V> vs;
  std::vector<double> vbytes;
  hipStream_t s0, s1;
  CK(hipStreamCreate(&s0));
  CK(hipStreamCreate(&s1));
  for (auto &s : sets) {
    std::vector<const float *> bv(s.b.p, s.b.p + 8);
    float *m = s.master;
    BucketPtrs bp = s.b;
    auto add = [&](std::string name, int nb, std::function<void()> f) {
      vs.push_back(V{s.name + " NB" + std::to_string(nb) + " " + name, f, {}});
      vbytes.push_back((nb + 2.0) * kN * 4);
    };
    for (int nb : {2, 8}) {
      add("prod", nb, [=]() { gp_bucket_sum_apply(m, bv.data(), nb, kN, nullptr); });
    }
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
  std::printf("%-34s %10s %10s %10s %8s\n", "arena / kernel", "med_ms", "min_ms", "GB/s", "frac8T");
  for (size_t i = 0; i < vs.size(); ++i) {
    auto &v = vs[i];
    const double bytes = vbytes[i];
    std::sort(v.ms.begin(), v.ms.end());
    const double med = v.ms[v.ms.size() / 2];
    const double gbs = bytes / (med * 1e-3) / 1e9;
    std::printf("%-34s %10.4f %10.4f %10.1f %8.4f\n", v.name.c_str(), med, v.ms[0], gbs, gbs / 8000.0);
  }
  return 0;
}
