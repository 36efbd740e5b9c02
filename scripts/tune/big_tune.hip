// big_tune.hip — bigger sweep chunks with shallower bursts, and a sweep whose
// last pass stores each tile as soon as it is summed (tuning harness, not
// product code; it #includes the product kernels).  Production (round 2): 96-MiB
// chunks = 10 LDS + 14 register tiles per block, bursts of 8 tiles.  Each
// launch pays a few us of ramp and drain (persist_tune.hip); larger chunks pay
// it fewer times: 18 register tiles (112 MiB) with bursts of 4 or 7, 16 (104
// MiB) with bursts of 2, against production at 1, 2 and 8 buckets, on whole
// chunks (bytes priced on the covered part), bit-checking every covered float.
// "fused last" writes each tile out in the last stream's pass instead of a
// separate write phase.  Pass 1 (profiles/r02/tune/big_tune.txt): 104 MiB with
// bursts of 2 ran +2-3 % at 8 buckets; fused last lost 5-12 %.  Pass 2 (this
// version) separates burst depth from chunk size: bursts of 1-8 at 96-120 MiB
// (profiles/r02/tune/big_tune2.txt): bursts of 2 at 96 MiB ran +2.3-3.5 % at 8
// buckets.  Pass 3 (this version): bursts of 1-3 at 64-96 MiB and 1-8 buckets,
// and the zero-input form (label NB0: out = 0.0f + b0, 2 streams)
// (profiles/r02/tune/big_tune3.txt): bursts of 2 +1.3-3.0 % at 3-8 buckets, tie
// at 2, -1 % at 1 and for the zero-input form.  Pass 4 (this version): the
// write phase throttled to WT stores in flight per wave (s_waitcnt vmcnt(WT)
// after each tile), since the read side gained from a narrower address window
// (profiles/r02/tune/big_tune4.txt: no effect).  Pass 5 (this version): burst
// depth and chunk size at 1-2 buckets, the zero-input form and the NB = 0 copy
// (a gather plan's dense runs; out = b0 here, so the copy reads another buffer)
// (profiles/r02/tune/big_tune5.txt: production best or tied).  Pass 6 (this
// version): tile width (sweep_u): 8 loads per wave as one contiguous 32-KiB
// run per CU (UU = 8, TG = 1) or four 8-KiB tiles (UU = 2, TG = 4)
// (profiles/r02/tune/big_tune6.txt): UU = 8, TG = 1 +0.4 % at 8 buckets, +2.2 %
// at 4 and +2 % at 2.  Pass 7: UU = 8 at 1-8 buckets, the zero-input form and
// the copy (big_tune7.txt: adopted at 2-8 buckets; 1 bucket tied or lost, the
// one-stream forms +-3 % by arena).  Pass 8 (this version, 4 arenas): the
// 64-MiB chunks after the big ones, 1 bucket with deeper 32-KiB bursts, and
// the one-stream forms again (big_tune8.txt: none adopted).  Pass 9 (this
// version): around the adopted 32-KiB shape -- write order, 88-104 MiB
// chunks, 40-KiB runs (10 block-strides per tile) (big_tune9.txt: the
// adopted shape is best or tied everywhere).  Pass 10 (this version): the
// one-stream forms (zero-input, copy) with 32-KiB tiles over 5 arenas, to
// settle big_tune7/8's +-3 % by arena (big_tune10.txt: zero-input +0.3 %,
// copy -0.8 % on average; production kept).  Pass 11 (this version): fewer
// LDS tiles and more register tiles in the same 96-MiB chunk (sweep_l)
// (big_tune11.txt: 4 LDS + 8 register tiles tie, 3 + 9 spill and lose 3-5 %,
// 2 + 10 lose 1 %: the LDS read-modify-write is not what bounds a pass).
// Pass 12 (this version): plain instead of non-temporal loads in that shape
// (big_tune12.txt: plain loads lose 5-10 %).
// Usage: big_tune [rounds] [arenas]
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


// The production sweep body with a zero-input option: ZIN sums out = 0.0f +
// b0 (+ b1 ...) (pass 0 adds its loads to +0.0f, so -0 -> +0 as after the
// memset the planned init replaces); otherwise out = in + b0 + ...
// vmcnt(N) alone (expcnt / lgkmcnt at their maxima: no wait on them)
constexpr int vmcnt_imm(int n) { return (n & 0xF) | (((n >> 4) & 3) << 14) | 0x70 | 0xF00; }

template <int NB, int RT, int TG, bool ZIN, bool FL = false, int WT = 0>
__global__ __launch_bounds__(kBlock) void sweep_lb(f4 *__restrict__ out, const f4 *__restrict__ in,
                                                   BucketPtrs b, size_t n4_tiles, size_t chunk) {
  constexpr int U = kPhaseU;
  constexpr int kT = kPhaseLdsTiles + RT;
  constexpr int S = ZIN ? NB : NB + 1;  // streams
  static_assert(kT % TG == 0, "whole bursts");
  __shared__ f4 res[kPhaseLdsF4];
  f4 keep[RT > 0 ? RT : 1][U];
  const f4 *src[S];
#pragma unroll
  for (int k = 0; k < S; ++k)
    src[k] = (!ZIN && k == 0) ? in : reinterpret_cast<const f4 *>(b.p[ZIN ? k : k - 1]);
  const size_t G = gridDim.x;
  const size_t lo = chunk * G * (size_t)kT * kPhaseTile;
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
          v[j][u] = ld_stream(src[k] + lo + ((size_t)(t0 + j) * G + blockIdx.x) * kPhaseTile +
                              threadIdx.x + u * kBlock);
#pragma unroll
      for (int j = 0; j < TG; ++j) {
        const int t = t0 + j;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const f4 first = ZIN ? f4(0.0f) + v[j][u] : v[j][u];
          if (FL && k == S - 1) {  // last pass: straight out
            const f4 s = k == 0 ? first
                                : (t < kPhaseLdsTiles ? res[t * kPhaseTile + u * kBlock + threadIdx.x]
                                                      : keep[t >= kPhaseLdsTiles ? t - kPhaseLdsTiles : 0][u]) +
                                      v[j][u];
            __builtin_nontemporal_store(s, out + lo + ((size_t)t * G + blockIdx.x) * kPhaseTile +
                                               threadIdx.x + u * kBlock);
          } else if (t < kPhaseLdsTiles) {
            f4 &r = res[t * kPhaseTile + u * kBlock + threadIdx.x];
            r = k == 0 ? first : r + v[j][u];
          } else {
            f4 &r = keep[t >= kPhaseLdsTiles ? t - kPhaseLdsTiles : 0][u];
            r = k == 0 ? first : r + v[j][u];
          }
        }
      }
    }
  }
  if (FL) return;
  __syncthreads();
#pragma unroll
  for (int t = 0; t < kT; ++t) {
    const size_t base = lo + ((size_t)t * G + blockIdx.x) * kPhaseTile + threadIdx.x;
#pragma unroll
    for (int u = 0; u < U; ++u)
      __builtin_nontemporal_store(t < kPhaseLdsTiles ? res[t * kPhaseTile + u * kBlock + threadIdx.x]
                                                     : keep[t >= kPhaseLdsTiles ? t - kPhaseLdsTiles : 0][u],
                                  out + base + u * kBlock);
    if (WT > 0) __builtin_amdgcn_s_waitcnt(vmcnt_imm(WT));  // at most WT stores in flight
  }
}

template <int NB, int RT, int TG, bool ZIN, bool FL = false, int WT = 0>
size_t launch_lb(float *out, const float *in, const BucketPtrs &b, bool run) {
  const size_t n4 = kN / 4;
  const size_t G = (size_t)num_cus();
  const size_t chunk_f4 = G * (size_t)(kPhaseLdsTiles + RT) * kPhaseTile;
  const size_t chunks = n4 / chunk_f4;
  if (run)
    for (size_t c = 0; c < chunks; ++c)
      hipLaunchKernelGGL((sweep_lb<NB, RT, TG, ZIN, FL, WT>), dim3((unsigned)G), dim3(kBlock), 0, 0,
                         reinterpret_cast<f4 *>(out), reinterpret_cast<const f4 *>(in), b, n4, c);
  return chunks * chunk_f4 * 4;
}


// Tile width as a parameter (UU block-strides of 4 KiB per tile; production
// UU = kPhaseU = 4): the same chunk and registers with wider tiles and fewer
// per burst, so a CU's burst is one contiguous 8 * 4-KiB run (UU = 8, TG = 1)
// instead of two 16-KiB tiles 4 MiB apart.
template <int NB, int RT, int TG, int UU, bool ZIN = false, bool REV = false>
__global__ __launch_bounds__(kBlock) void sweep_u(f4 *__restrict__ out, const f4 *__restrict__ in,
                                                  BucketPtrs b, size_t n4_tiles, size_t chunk) {
  constexpr int kTile = kBlock * UU;
  constexpr int kLds = kPhaseLdsF4 / kTile;
  static_assert(kLds * kTile == kPhaseLdsF4, "whole LDS tiles");
  constexpr int kT = kLds + RT;
  constexpr int S = ZIN ? NB : NB + 1;
  static_assert(kT % TG == 0, "whole bursts");
  __shared__ f4 res[kPhaseLdsF4];
  f4 keep[RT][UU];
  const f4 *src[S];
#pragma unroll
  for (int k = 0; k < S; ++k)
    src[k] = (!ZIN && k == 0) ? in : reinterpret_cast<const f4 *>(b.p[ZIN ? k : (k > 0 ? k - 1 : 0)]);
  const size_t G = gridDim.x;
  const size_t lo = chunk * G * (size_t)kT * kTile;
  if (lo >= n4_tiles) return;
#pragma unroll
  for (int k = 0; k < S; ++k) {
#pragma unroll
    for (int t0 = 0; t0 < kT; t0 += TG) {
      f4 v[TG][UU];
#pragma unroll
      for (int j = 0; j < TG; ++j)
#pragma unroll
        for (int u = 0; u < UU; ++u)
          v[j][u] = ld_stream(src[k] + lo + ((size_t)(t0 + j) * G + blockIdx.x) * kTile + threadIdx.x + u * kBlock);
#pragma unroll
      for (int j = 0; j < TG; ++j) {
        const int t = t0 + j;
#pragma unroll
        for (int u = 0; u < UU; ++u) {
          const f4 first = ZIN ? f4(0.0f) + v[j][u] : v[j][u];
          if (t < kLds) {
            f4 &r = res[t * kTile + u * kBlock + threadIdx.x];
            r = k == 0 ? first : r + v[j][u];
          } else {
            f4 &r = keep[t >= kLds ? t - kLds : 0][u];
            r = k == 0 ? first : r + v[j][u];
          }
        }
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int t_ = 0; t_ < kT; ++t_) {
    const int t = REV ? kT - 1 - t_ : t_;  // REV: register tiles out first
    const size_t base = lo + ((size_t)t * G + blockIdx.x) * kTile + threadIdx.x;
#pragma unroll
    for (int u = 0; u < UU; ++u)
      __builtin_nontemporal_store(t < kLds ? res[t * kTile + u * kBlock + threadIdx.x] : keep[t >= kLds ? t - kLds : 0][u],
                                  out + base + u * kBlock);
  }
}

template <int NB, int RT, int TG, int UU, bool ZIN = false, bool REV = false>
size_t launch_u(float *out, const float *in, const BucketPtrs &b, bool run) {
  const size_t n4 = kN / 4;
  const size_t G = (size_t)num_cus();
  const size_t chunk_f4 = G * (size_t)(kPhaseLdsF4 / (kBlock * UU) + RT) * kBlock * UU;
  const size_t chunks = n4 / chunk_f4;
  if (run)
    for (size_t c = 0; c < chunks; ++c)
      hipLaunchKernelGGL((sweep_u<NB, RT, TG, UU, ZIN, REV>), dim3((unsigned)G), dim3(kBlock), 0, 0,
                         reinterpret_cast<f4 *>(out), reinterpret_cast<const f4 *>(in), b, n4, c);
  return chunks * chunk_f4 * 4;
}


// LDS tiles as a parameter (NL of UU * 4 KiB; production: 160 KiB = 5 x 32 KiB
// beside 7 register tiles): the same 96-MiB chunk with fewer tiles parked in
// LDS and more in registers, so each pass does less LDS read-modify-write.
template <int NB, int RT, int TG, int UU, int NL, bool PL = false>
__global__ __launch_bounds__(kBlock) void sweep_l(f4 *__restrict__ out, const f4 *__restrict__ in,
                                                  BucketPtrs b, size_t n4_tiles, size_t chunk) {
  constexpr int kTile = kBlock * UU;
  constexpr int kT = NL + RT;
  constexpr int S = NB + 1;
  static_assert(kT % TG == 0, "whole bursts");
  __shared__ f4 res[NL > 0 ? NL * kTile : 1];
  f4 keep[RT][UU];
  const f4 *src[S];
#pragma unroll
  for (int k = 0; k < S; ++k) src[k] = k == 0 ? in : reinterpret_cast<const f4 *>(b.p[k - 1]);
  const size_t G = gridDim.x;
  const size_t lo = chunk * G * (size_t)kT * kTile;
  if (lo >= n4_tiles) return;
#pragma unroll
  for (int k = 0; k < S; ++k) {
#pragma unroll
    for (int t0 = 0; t0 < kT; t0 += TG) {
      f4 v[TG][UU];
#pragma unroll
      for (int j = 0; j < TG; ++j)
#pragma unroll
        for (int u = 0; u < UU; ++u)
          v[j][u] = PL ? src[k][lo + ((size_t)(t0 + j) * G + blockIdx.x) * kTile + threadIdx.x + u * kBlock]
                       : ld_stream(src[k] + lo + ((size_t)(t0 + j) * G + blockIdx.x) * kTile + threadIdx.x + u * kBlock);
#pragma unroll
      for (int j = 0; j < TG; ++j) {
        const int t = t0 + j;
#pragma unroll
        for (int u = 0; u < UU; ++u) {
          if (t < NL) {
            f4 &r = res[t * kTile + u * kBlock + threadIdx.x];
            r = k == 0 ? v[j][u] : r + v[j][u];
          } else {
            f4 &r = keep[t >= NL ? t - NL : 0][u];
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
    for (int u = 0; u < UU; ++u)
      __builtin_nontemporal_store(t < NL ? res[t * kTile + u * kBlock + threadIdx.x] : keep[t >= NL ? t - NL : 0][u],
                                  out + base + u * kBlock);
  }
}

template <int NB, int RT, int TG, int UU, int NL, bool PL = false>
size_t launch_l(float *out, const float *in, const BucketPtrs &b, bool run) {
  const size_t n4 = kN / 4;
  const size_t G = (size_t)num_cus();
  const size_t chunk_f4 = G * (size_t)(NL + RT) * kBlock * UU;
  const size_t chunks = n4 / chunk_f4;
  if (run)
    for (size_t c = 0; c < chunks; ++c)
      hipLaunchKernelGGL((sweep_l<NB, RT, TG, UU, NL, PL>), dim3((unsigned)G), dim3(kBlock), 0, 0,
                         reinterpret_cast<f4 *>(out), reinterpret_cast<const f4 *>(in), b, n4, c);
  return chunks * chunk_f4 * 4;
}

template <int NB, int RT, int TG, int UU, int NL>
void report_l(const char *name) {
  hipFuncAttributes a;
  CK(hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&sweep_l<NB, RT, TG, UU, NL>)));
  std::printf("%-26s regs %d  scratch %zu B/lane  lds %zu B\n", name, a.numRegs, a.localSizeBytes, a.sharedSizeBytes);
}

template <int NB, int RT, int TG, bool ZIN, bool FL = false>
void report(const char *name) {
  hipFuncAttributes a;
  CK(hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&sweep_lb<NB, RT, TG, ZIN, FL>)));
  std::printf("%-22s regs %d  scratch %zu B/lane\n", name, a.numRegs, a.localSizeBytes);
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
    std::function<size_t(float *, const BucketPtrs &, bool)> run;
  };
  auto prod_sum = [](int nb) {
    return [nb](float *m, const BucketPtrs &b, bool run) {
      std::vector<const float *> bv(b.p, b.p + nb);
      if (run) gp_bucket_sum_apply(m, bv.data(), nb, kN, nullptr);
      return kN;
    };
  };
#define LB(NB, RT, TG, FL) [](float *m, const BucketPtrs &b, bool r) { return launch_lb<NB, RT, TG, false, FL>(m, m, b, r); }
  auto prod_zin = [](float *m, const BucketPtrs &b, bool run) {
    if (run) launch_bucket_sum_nb<1, true>(m, nullptr, b, kN, nullptr);
    return kN;
  };
#define LBW(NB, RT, TG, WT) [](float *m, const BucketPtrs &b, bool r) { return launch_lb<NB, RT, TG, false, false, WT>(m, m, b, r); }
#define LBZ(RT, TG, WT) [](float *m, const BucketPtrs &b, bool r) { return launch_lb<1, RT, TG, true, false, WT>(m, m, b, r); }
#define LB0(RT, TG) [](float *m, const BucketPtrs &b, bool r) { return launch_lb<0, RT, TG, false, false, 0>(m, b.p[0], b, r); }
  auto prod_copy = [](float *m, const BucketPtrs &b, bool run) {
    if (run) launch_bucket_sum_nb<0>(m, b.p[0], b, kN, nullptr);
    return kN;
  };
#define LU(NB, RT, TG, UU) [](float *m, const BucketPtrs &b, bool r) { return launch_u<NB, RT, TG, UU>(m, m, b, r); }
#define LUZ(RT, TG, UU) [](float *m, const BucketPtrs &b, bool r) { return launch_u<1, RT, TG, UU, true>(m, m, b, r); }
#define LU0(RT, TG, UU) [](float *m, const BucketPtrs &b, bool r) { return launch_u<0, RT, TG, UU>(m, b.p[0], b, r); }
#define LUR(NB, RT, TG, UU) [](float *m, const BucketPtrs &b, bool r) { return launch_u<NB, RT, TG, UU, false, true>(m, m, b, r); }
#define LL(NB, RT, NL) [](float *m, const BucketPtrs &b, bool r) { return launch_l<NB, RT, 1, 8, NL>(m, m, b, r); }
#define LLP(NB, RT, NL) [](float *m, const BucketPtrs &b, bool r) { return launch_l<NB, RT, 1, 8, NL, true>(m, m, b, r); }
  std::vector<V> kinds = {
      {"prod (32-KiB tiles + 64 MiB)", 8, prod_sum(8)},
      {"L5 R7 nt loads (prod shape)", 8, LL(8, 7, 5)},
      {"L5 R7 plain loads", 8, LLP(8, 7, 5)},
      {"prod (32-KiB tiles + tile-major)", 2, prod_sum(2)},
      {"L5 R7 nt loads (prod shape)", 2, LL(2, 7, 5)},
      {"L5 R7 plain loads", 2, LLP(2, 7, 5)},
  };
#undef LLP
#undef LL
#undef LUR
#undef LUZ
#undef LU0
#undef LU
#undef LB0
#undef LBW
#undef LBZ
#undef LB
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
                     (v.nb == 0 ? 2.0 : v.nb + 2.0) * covered * 4, {}});
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
