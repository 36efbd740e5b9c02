// r6_multichunk_tune.hip — does a sweep launch that sums P chunks back to back
// (no grid barrier between them) beat one launch per chunk?  Tuning harness,
// not product code; it #includes the product kernel file.
//
// Why: at 2 buckets (configs[1]) a 96-MiB chunk takes ~61 us and the sum runs
// at 94-95 % of the box's two-rate model, against 98-99 % at 8 buckets
// (146 us a chunk): a fixed ~3 us per launch (ramp-up of the first loads, the
// drain of the last writes) weighs 2.5x more.  P chunks per launch pay it once
// per P chunks; the price is that blocks drift apart between chunks (a fast
// block reads chunk c+1 while a slow one still writes chunk c).
//
// Each variant is checked bit for bit against the production launch sequence
// on the chunks it covers, then all variants are timed in interleaved rounds
// on the same buffers (median per variant).  Usage:
//   r6_multichunk_tune [rounds]      (1M x 1024 fp32 shard; NB = 2 and 8)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include \
//   scripts/tune/r6_multichunk_tune.hip geeps_amd/csrc/gp_sort.hip -o build/probe/r6_multichunk_tune
// (-DR6_CHUNK_SIZES: the second pass, one chunk per launch at other chunk
// sizes, i.e. register tile counts).
#include "../../geeps_amd/csrc/gp_reduce.hip"

#include <algorithm>
#include <cstdlib>
#include <functional>

#define CK(x)                                                                                       \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) {                                                                         \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));       \
      std::exit(2);                                                                                 \
    }                                                                                               \
  } while (0)

namespace {

// bucket_sum_sweep_kernel with an outer loop over P consecutive chunks
// (chunk index = launch index * P + c); same per-chunk body.
template <int NB, int RT, int TG, int U, int P>
__global__ __launch_bounds__(kBlock) void multi_sweep_kernel(f4 *__restrict__ out, const f4 *__restrict__ in,
                                                             BucketPtrs b, size_t n4_tiles, size_t launch) {
  constexpr int kTile = kBlock * U;
  constexpr int kLds = kPhaseLdsF4 / kTile;
  constexpr int kT = kLds + RT;
  constexpr int S = NB + 1;
  static_assert(kT % TG == 0, "whole bursts");
  __shared__ f4 res[kPhaseLdsF4];
  f4 keep[RT][U];
  const f4 *src[S];
#pragma unroll
  for (int k = 0; k < S; ++k) src[k] = k == 0 ? in : reinterpret_cast<const f4 *>(b.p[k - 1]);
  const size_t G = gridDim.x;
  for (int c = 0; c < P; ++c) {
    const size_t lo = (launch * P + c) * G * (size_t)kT * kTile;
    if (lo >= n4_tiles) return;
#pragma unroll
    for (int k = 0; k < S; ++k) {
#pragma unroll
      for (int t0 = 0; t0 < kT; t0 += TG) {
        f4 v[TG][U];
#pragma unroll
        for (int j = 0; j < TG; ++j)
#pragma unroll
          for (int u = 0; u < U; ++u)
            v[j][u] = ld_stream(src[k] + lo + ((size_t)(t0 + j) * G + blockIdx.x) * kTile + threadIdx.x + u * kBlock);
#pragma unroll
        for (int j = 0; j < TG; ++j) {
          const int t = t0 + j;
#pragma unroll
          for (int u = 0; u < U; ++u) {
            if (t < kLds) {
              f4 &r = res[t * kTile + u * kBlock + threadIdx.x];
              r = k == 0 ? v[j][u] : r + v[j][u];
            } else {
              f4 &r = keep[t >= kLds ? t - kLds : 0][u];
              r = k == 0 ? v[j][u] : r + v[j][u];
            }
          }
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < kT; ++t) {
      const size_t base = lo + ((size_t)t * G + blockIdx.x) * kTile + threadIdx.x;
#pragma unroll
      for (int u = 0; u < U; ++u)
        __builtin_nontemporal_store(t < kLds ? res[t * kTile + u * kBlock + threadIdx.x] : keep[t >= kLds ? t - kLds : 0][u],
                                    out + base + u * kBlock);
    }
    __syncthreads();  // the block's LDS slots are reused by the next chunk
  }
}

struct Variant {
  std::string name;
  size_t chunk_f4;  // per launch, all blocks
  std::function<void(f4 *, const f4 *, const BucketPtrs &, size_t, size_t, hipStream_t)> run;  // launch l
};

template <int NB, int RT, int TG, int U, int P>
Variant make(const char *tag) {
  const size_t G = (size_t)num_cus();
  constexpr int kT = kPhaseLdsF4 / (kBlock * U) + RT;
  Variant v;
  v.name = std::string("NB") + std::to_string(NB) + " " + tag + " RT" + std::to_string(RT) + " TG" + std::to_string(TG) +
           " U" + std::to_string(U) + " P" + std::to_string(P);
  v.chunk_f4 = G * (size_t)kT * kBlock * U * P;
  v.run = [G](f4 *out, const f4 *in, const BucketPtrs &b, size_t n4, size_t l, hipStream_t s) {
    hipLaunchKernelGGL((multi_sweep_kernel<NB, RT, TG, U, P>), dim3((unsigned)G), dim3(kBlock), 0, s, out, in, b, n4, l);
  };
  return v;
}

}  // namespace

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 7;
  const size_t n = (size_t)1 << 30;  // 1M x 1024 floats (4 GiB)
  const size_t n4 = n / 4;
  std::vector<f4 *> bk(8);
  for (auto &p : bk) CK(hipMalloc(&p, n * 4));
  f4 *master, *check;
  CK(hipMalloc(&master, n * 4));
  CK(hipMalloc(&check, n * 4));
  // fill with small integers-as-floats patterns that differ per buffer
  for (int k = 0; k < 8; ++k) {
    std::vector<float> h(1 << 20);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * (k + 3) + k) % 1000) * 0.001f - 0.5f;
    for (size_t off = 0; off < n; off += h.size()) CK(hipMemcpy((float *)bk[k] + off, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  }
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int NB : {2, 8}) {
    BucketPtrs b = {};
    for (int k = 0; k < NB; ++k) b.p[k] = reinterpret_cast<const float *>(bk[k]);
    std::vector<Variant> vs;
#ifdef R6_CHUNK_SIZES
    // round 6, second pass: one chunk per launch, chunk size by register tiles
    if (NB == 2) {
      vs.push_back(make<2, 7, 1, 8, 1>("prod shape"));
      vs.push_back(make<2, 3, 1, 8, 1>("64 MiB"));
      vs.push_back(make<2, 9, 1, 8, 1>("112 MiB"));
      vs.push_back(make<2, 11, 1, 8, 1>("128 MiB"));
      vs.push_back(make<2, 13, 1, 8, 1>("144 MiB"));
    } else {
      vs.push_back(make<8, 7, 1, 8, 1>("prod shape"));
      vs.push_back(make<8, 8, 1, 8, 1>("104 MiB"));
      vs.push_back(make<8, 9, 1, 8, 1>("112 MiB"));
      vs.push_back(make<8, 11, 1, 8, 1>("128 MiB"));
    }
#else
    if (NB == 2) {
      vs.push_back(make<2, 7, 1, 8, 1>("prod shape"));
      vs.push_back(make<2, 7, 1, 8, 2>("prod shape"));
      vs.push_back(make<2, 7, 1, 8, 4>("prod shape"));
      vs.push_back(make<2, 14, 8, 4, 1>("16K tiles"));
      vs.push_back(make<2, 14, 8, 4, 2>("16K tiles"));
      vs.push_back(make<2, 7, 2, 8, 2>("burst2"));
    } else {
      vs.push_back(make<8, 7, 1, 8, 1>("prod shape"));
      vs.push_back(make<8, 7, 1, 8, 2>("prod shape"));
      vs.push_back(make<8, 7, 1, 8, 3>("prod shape"));
    }
#endif
    // bit check against production (gp_bucket_sum_into over the same prefix)
    for (auto &v : vs) {
      const size_t launches = n4 / v.chunk_f4, covered = launches * v.chunk_f4;
      CK(hipMemset(master, 0, n * 4));
      CK(hipMemset(check, 0, n * 4));
      const float *bp[8];
      for (int k = 0; k < NB; ++k) bp[k] = reinterpret_cast<const float *>(bk[k]);
      if (gp_bucket_sum_into(reinterpret_cast<float *>(check), reinterpret_cast<float *>(check), bp, NB, covered * 4,
                             s) != GP_OK) {
        std::fprintf(stderr, "prod failed: %s\n", gp_last_error());
        return 2;
      }
      for (size_t l = 0; l < launches; ++l) v.run(master, master, b, covered, l, s);
      CK(hipStreamSynchronize(s));
      std::vector<uint32_t> a(1 << 22), c(1 << 22);
      size_t bad = 0;
      for (size_t off = 0; off < covered * 4; off += a.size()) {
        const size_t m = std::min(a.size(), covered * 4 - off);
        CK(hipMemcpy(a.data(), (float *)master + off, m * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(c.data(), (float *)check + off, m * 4, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < m; ++i) bad += a[i] != c[i];
      }
      std::printf("%-34s covers %zu floats (%.1f%%): %zu mismatches\n", v.name.c_str(), covered * 4,
                  100.0 * covered / n4, bad);
    }
    std::vector<std::vector<double>> ms(vs.size());
    for (int r = 0; r < rounds; ++r)
      for (size_t i = 0; i < vs.size(); ++i) {
        auto &v = vs[i];
        const size_t launches = n4 / v.chunk_f4, covered = launches * v.chunk_f4;
        for (size_t l = 0; l < launches; ++l) v.run(master, master, b, covered, l, s);  // warm
        CK(hipEventRecord(e0, s));
        for (int rep = 0; rep < 3; ++rep)
          for (size_t l = 0; l < launches; ++l) v.run(master, master, b, covered, l, s);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float t = 0;
        CK(hipEventElapsedTime(&t, e0, e1));
        ms[i].push_back(t / 3 / covered * n4);  // scaled to the whole 4-GiB shard
      }
    std::printf("%-34s %10s %10s %10s %8s\n", "variant (NB, shape, chunks/launch)", "med_ms", "min_ms", "GB/s", "frac8T");
    for (size_t i = 0; i < vs.size(); ++i) {
      auto m = ms[i];
      std::sort(m.begin(), m.end());
      const double med = m[m.size() / 2], bytes = (double)(NB + 2) * n * 4;
      std::printf("%-34s %10.4f %10.4f %10.1f %8.4f\n", vs[i].name.c_str(), med, m[0], bytes / med / 1e6,
                  bytes / med / 1e6 / 8000.0);
    }
  }
  return 0;
}
