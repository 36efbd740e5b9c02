// bucket_tune.hip — variant sweep for the N-way bucket-sum kernel (tuning
// harness, not product code).  Interleaved rounds in ONE process; reports the
// median per variant.  Usage: bucket_tune [rows] [width] [buckets] [rounds]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e = (x);                                                     \
    if (e != hipSuccess) {                                                  \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,         \
                   hipGetErrorString(e));                                   \
      std::exit(2);                                                         \
    }                                                                       \
  } while (0)

constexpr int kB = 256;
struct Ptrs {
  const f4 *p[16];
};

template <int NB, int U, bool NTB, bool NTM, bool NTS>
__global__ __launch_bounds__(kB) void bsum(f4 *__restrict__ out, const f4 *__restrict__ in,
                                           Ptrs b, size_t n4) {
  const size_t tile = (size_t)kB * U;
  const size_t stride = (size_t)gridDim.x * tile;
  size_t base = (size_t)blockIdx.x * tile + threadIdx.x;
  for (; base + (U - 1) * kB < n4; base += stride) {
    f4 acc[U];
    f4 v[NB][U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      acc[u] = NTM ? __builtin_nontemporal_load(in + base + u * kB) : in[base + u * kB];
#pragma unroll
    for (int k = 0; k < NB; ++k)
#pragma unroll
      for (int u = 0; u < U; ++u)
        v[k][u] = NTB ? __builtin_nontemporal_load(b.p[k] + base + u * kB) : b.p[k][base + u * kB];
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int k = 0; k < NB; ++k) acc[u] += v[k][u];
      if (NTS)
        __builtin_nontemporal_store(acc[u], out + base + u * kB);
      else
        out[base + u * kB] = acc[u];
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const size_t i = base + u * kB;
    if (i < n4) {
      f4 acc = in[i];
#pragma unroll
      for (int k = 0; k < NB; ++k) acc += b.p[k][i];
      out[i] = acc;
    }
  }
}

// Block-contiguous form: each block owns a contiguous chunk of the array.
template <int NB, bool NTB>
__global__ __launch_bounds__(kB) void bsum_chunk(f4 *__restrict__ out, const f4 *__restrict__ in,
                                                 Ptrs b, size_t n4, size_t chunk) {
  const size_t lo = (size_t)blockIdx.x * chunk;
  const size_t hi = lo + chunk < n4 ? lo + chunk : n4;
  for (size_t i = lo + threadIdx.x; i < hi; i += kB) {
    f4 acc = in[i];
    f4 v[NB];
#pragma unroll
    for (int k = 0; k < NB; ++k) v[k] = NTB ? __builtin_nontemporal_load(b.p[k] + i) : b.p[k][i];
#pragma unroll
    for (int k = 0; k < NB; ++k) acc += v[k];
    out[i] = acc;
  }
}


// General form: block size BS, U tiles per thread, optional XCD-contiguous tile remap.
template <int NB, int U, int BS, bool XCD>
__global__ __launch_bounds__(BS) void bsum2(f4 *__restrict__ out, const f4 *__restrict__ in,
                                            Ptrs b, size_t n4) {
  const size_t tile = (size_t)BS * U;
  const size_t stride = (size_t)gridDim.x * tile;
  unsigned lb = blockIdx.x;
  if (XCD) {  // blocks b, b+8, ... share an XCD: give each XCD a contiguous slice of the window
    const unsigned g8 = gridDim.x / 8;
    lb = (blockIdx.x % 8) * g8 + blockIdx.x / 8;
  }
  size_t base = (size_t)lb * tile + threadIdx.x;
  for (; base + (U - 1) * BS < n4; base += stride) {
    f4 acc[U];
    f4 v[NB][U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = in[base + u * BS];
#pragma unroll
    for (int k = 0; k < NB; ++k)
#pragma unroll
      for (int u = 0; u < U; ++u) v[k][u] = __builtin_nontemporal_load(b.p[k] + base + u * BS);
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int k = 0; k < NB; ++k) acc[u] += v[k][u];
      out[base + u * BS] = acc[u];
    }
  }
  for (int u = 0; u < U; ++u) {
    const size_t i = base + u * BS;
    if (i < n4) {
      f4 acc = in[i];
      for (int k = 0; k < NB; ++k) acc += b.p[k][i];
      out[i] = acc;
    }
  }
}

// Software-pipelined: the next tile's loads are issued before this tile's store.
template <int NB>
__global__ __launch_bounds__(kB) void bsum_pipe(f4 *__restrict__ out, const f4 *__restrict__ in,
                                                Ptrs b, size_t n4) {
  const size_t stride = (size_t)gridDim.x * kB;
  size_t i = (size_t)blockIdx.x * kB + threadIdx.x;
  if (i >= n4) return;
  f4 acc = in[i];
  f4 v[NB];
#pragma unroll
  for (int k = 0; k < NB; ++k) v[k] = __builtin_nontemporal_load(b.p[k] + i);
  for (;;) {
    const size_t j = i + stride;
    f4 acc2 = acc, v2[NB];
    const bool more = j < n4;
    if (more) {
      acc2 = in[j];
#pragma unroll
      for (int k = 0; k < NB; ++k) v2[k] = __builtin_nontemporal_load(b.p[k] + j);
    }
#pragma unroll
    for (int k = 0; k < NB; ++k) acc += v[k];
    out[i] = acc;
    if (!more) break;
    acc = acc2;
#pragma unroll
    for (int k = 0; k < NB; ++k) v[k] = v2[k];
    i = j;
  }
}

// Ceiling probes: 9 read streams with no store (store guarded by a runtime flag
// that is never set), and a 1-stream write.
template <int NB>
__global__ __launch_bounds__(kB) void read_only(f4 *__restrict__ out, const f4 *__restrict__ in,
                                                Ptrs b, size_t n4, int flag) {
  const size_t stride = (size_t)gridDim.x * kB;
  f4 tot = {0, 0, 0, 0};
  for (size_t i = (size_t)blockIdx.x * kB + threadIdx.x; i < n4; i += stride) {
    f4 acc = __builtin_nontemporal_load(in + i);
#pragma unroll
    for (int k = 0; k < NB; ++k) acc += __builtin_nontemporal_load(b.p[k] + i);
    tot += acc;
  }
  if (flag) out[blockIdx.x * kB + threadIdx.x] = tot;
}

__global__ void write_only(f4 *__restrict__ out, size_t n4) {
  const size_t stride = (size_t)gridDim.x * kB;
  const f4 z = {1, 2, 3, 4};
  for (size_t i = (size_t)blockIdx.x * kB + threadIdx.x; i < n4; i += stride) out[i] = z;
}

__global__ void copy_nt4(f4 *__restrict__ out, const f4 *__restrict__ in, size_t n4) {
  const size_t stride = (size_t)gridDim.x * kB * 4;
  size_t i = (size_t)blockIdx.x * kB * 4 + threadIdx.x;
  for (; i + 3 * kB < n4; i += stride) {
    f4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(in + i + u * kB);
#pragma unroll
    for (int u = 0; u < 4; ++u) out[i + u * kB] = v[u];
  }
}


// Store cache-policy probe: the result store issued with explicit gfx950 cache
// bits (sc0 / sc1 / nt) through inline asm; loads as in production.
template <int U, int POL>
__global__ __launch_bounds__(kB) void bsum_pol(f4 *__restrict__ out, const f4 *__restrict__ in,
                                               Ptrs b, size_t n4) {
  constexpr int NB = 8;
  const size_t tile = (size_t)kB * U;
  const size_t stride = (size_t)gridDim.x * tile;
  size_t base = (size_t)blockIdx.x * tile + threadIdx.x;
  for (; base + (U - 1) * kB < n4; base += stride) {
    f4 acc[U];
    f4 v[NB][U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = in[base + u * kB];
#pragma unroll
    for (int k = 0; k < NB; ++k)
#pragma unroll
      for (int u = 0; u < U; ++u) v[k][u] = __builtin_nontemporal_load(b.p[k] + base + u * kB);
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int k = 0; k < NB; ++k) acc[u] += v[k][u];
      f4 *dst = out + base + u * kB;
      if (POL == 1) asm volatile("global_store_dwordx4 %0, %1, off sc1" :: "v"(dst), "v"(acc[u]) : "memory");
      if (POL == 2) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" :: "v"(dst), "v"(acc[u]) : "memory");
      if (POL == 3) asm volatile("global_store_dwordx4 %0, %1, off nt sc1" :: "v"(dst), "v"(acc[u]) : "memory");
      if (POL == 4) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" :: "v"(dst), "v"(acc[u]) : "memory");
      if (POL == 5) asm volatile("global_store_dwordx4 %0, %1, off nt" :: "v"(dst), "v"(acc[u]) : "memory");
    }
  }
}


// Diagnostic: same loads and adds, but the store goes to a 64 KiB L2-resident
// window (wrong results) — separates the HBM write cost from everything else.
template <int U>
__global__ __launch_bounds__(kB) void bsum_fakestore(f4 *__restrict__ out, const f4 *__restrict__ in,
                                                     Ptrs b, size_t n4) {
  constexpr int NB = 8;
  const size_t tile = (size_t)kB * U;
  const size_t stride = (size_t)gridDim.x * tile;
  size_t base = (size_t)blockIdx.x * tile + threadIdx.x;
  for (; base + (U - 1) * kB < n4; base += stride) {
    f4 acc[U];
    f4 v[NB][U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = in[base + u * kB];
#pragma unroll
    for (int k = 0; k < NB; ++k)
#pragma unroll
      for (int u = 0; u < U; ++u) v[k][u] = __builtin_nontemporal_load(b.p[k] + base + u * kB);
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int k = 0; k < NB; ++k) acc[u] += v[k][u];
      out[(base + u * kB) & 4095] = acc[u];
    }
  }
}

// R contiguous regions swept concurrently: block b works in region b % R.
template <int U, int R>
__global__ __launch_bounds__(kB) void bsum_regions(f4 *__restrict__ out, const f4 *__restrict__ in,
                                                   Ptrs b, size_t n4) {
  constexpr int NB = 8;
  const size_t per = (n4 + R - 1) / R;
  const unsigned reg = blockIdx.x % R, gb = gridDim.x / R, lb = blockIdx.x / R;
  const size_t lo = reg * per, hi = (lo + per < n4) ? lo + per : n4;
  const size_t tile = (size_t)kB * U;
  const size_t stride = (size_t)gb * tile;
  size_t base = lo + (size_t)lb * tile + threadIdx.x;
  for (; base + (U - 1) * kB < hi; base += stride) {
    f4 acc[U];
    f4 v[NB][U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = in[base + u * kB];
#pragma unroll
    for (int k = 0; k < NB; ++k)
#pragma unroll
      for (int u = 0; u < U; ++u) v[k][u] = __builtin_nontemporal_load(b.p[k] + base + u * kB);
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int k = 0; k < NB; ++k) acc[u] += v[k][u];
      out[base + u * kB] = acc[u];
    }
  }
}

__global__ void copy_k(f4 *__restrict__ out, const f4 *__restrict__ in, size_t n4) {
  const size_t stride = (size_t)gridDim.x * kB;
  for (size_t i = (size_t)blockIdx.x * kB + threadIdx.x; i < n4; i += stride) out[i] = in[i];
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
  const size_t rows = argc > 1 ? std::strtoull(argv[1], 0, 10) : (1ull << 20);
  const size_t width = argc > 2 ? std::strtoull(argv[2], 0, 10) : 1024;
  const int NBk = argc > 3 ? std::atoi(argv[3]) : 8;
  const int rounds = argc > 4 ? std::atoi(argv[4]) : 5;
  if (NBk != 8) {
    std::fprintf(stderr, "this harness is specialised for 8 buckets\n");
    return 1;
  }
  const size_t n = rows * width, n4 = n / 4;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  std::vector<float *> bk(NBk);
  float *master = nullptr, *scratch = nullptr;
  for (auto &p : bk) CK(hipMalloc(&p, n * 4));
  CK(hipMalloc(&master, n * 4));
  CK(hipMalloc(&scratch, n * 4));
  for (int k = 0; k < NBk; ++k) fill_k<<<4096, 256>>>(bk[k], n, 1000 + k);
  fill_k<<<4096, 256>>>(master, n, 77);
  CK(hipDeviceSynchronize());
  Ptrs P{};
  for (int k = 0; k < NBk; ++k) P.p[k] = reinterpret_cast<const f4 *>(bk[k]);
  f4 *m4 = reinterpret_cast<f4 *>(master);

  struct V {
    std::string name;
    double bytes;
    std::function<void()> run;
    std::vector<float> ms;
  };
  std::vector<V> vs;
  const double sum_bytes = (double)(NBk + 2) * n * 4;
  auto grid = [&](int per_cu, int U) {
    size_t tiles = (n4 + (size_t)kB * U - 1) / ((size_t)kB * U);
    size_t g = (size_t)cus * per_cu;
    return (unsigned)std::min(tiles, g);
  };
#define ADD(NAME, BYTES, ...) vs.push_back(V{NAME, BYTES, [&]() { __VA_ARGS__; }, {}})
  f4 *s4 = reinterpret_cast<f4 *>(scratch);
  (void)s4;
  // one arena, buckets then master (the production layout)
  char *ar = nullptr;
  CK(hipMalloc(&ar, 9 * n * 4));
  Ptrs A{};
  for (int k = 0; k < 8; ++k) {
    A.p[k] = reinterpret_cast<const f4 *>(ar + (size_t)k * n * 4);
    fill_k<<<4096, 256>>>(reinterpret_cast<float *>(ar + (size_t)k * n * 4), n, 1000 + k);
  }
  f4 *am = reinterpret_cast<f4 *>(ar + (size_t)8 * n * 4);
  fill_k<<<4096, 256>>>(reinterpret_cast<float *>(am), n, 77);
  CK(hipDeviceSynchronize());
  ADD("arena U4 pc2 (prod)", sum_bytes, (bsum<8, 4, true, false, false><<<grid(2, 4), kB>>>(am, am, A, n4)));
  ADD("arena U1 pc8", sum_bytes, (bsum<8, 1, true, false, false><<<grid(8, 1), kB>>>(am, am, A, n4)));
  ADD("arena U2 pc1", sum_bytes, (bsum<8, 2, true, false, false><<<grid(1, 2), kB>>>(am, am, A, n4)));
  ADD("arena U2 pc2", sum_bytes, (bsum<8, 2, true, false, false><<<grid(2, 2), kB>>>(am, am, A, n4)));
  ADD("arena U2 pc4", sum_bytes, (bsum<8, 2, true, false, false><<<grid(4, 2), kB>>>(am, am, A, n4)));
  ADD("arena U4 pc1", sum_bytes, (bsum<8, 4, true, false, false><<<grid(1, 4), kB>>>(am, am, A, n4)));
  ADD("arena U4 pc3", sum_bytes, (bsum<8, 4, true, false, false><<<grid(3, 4), kB>>>(am, am, A, n4)));
  ADD("arena U4 pc4", sum_bytes, (bsum<8, 4, true, false, false><<<grid(4, 4), kB>>>(am, am, A, n4)));
  ADD("arena U8 pc1", sum_bytes, (bsum<8, 8, true, false, false><<<grid(1, 8), kB>>>(am, am, A, n4)));
  ADD("arena U4 pc2 ntS", sum_bytes, (bsum<8, 4, true, false, true><<<grid(2, 4), kB>>>(am, am, A, n4)));
  ADD("arena U4 pc2 plain loads", sum_bytes, (bsum<8, 4, false, false, false><<<grid(2, 4), kB>>>(am, am, A, n4)));
  ADD("arena read9 only pc8", 9.0 * n * 4, (read_only<8><<<grid(8, 1), kB>>>(am, am, A, n4, 0)));

  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (auto &v : vs) v.run();  // warm-up
  CK(hipDeviceSynchronize());
  for (int r = 0; r < rounds; ++r) {
    for (auto &v : vs) {
      CK(hipEventRecord(a));
      v.run();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      v.ms.push_back(ms);
    }
    std::fprintf(stderr, "round %d done\n", r);
  }
  std::printf("%-44s %10s %10s %10s %8s\n", "variant", "med_ms", "min_ms", "GB/s", "frac8T");
  for (auto &v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const double med = v.ms[v.ms.size() / 2];
    const double gbs = v.bytes / (med * 1e-3) / 1e9;
    std::printf("%-44s %10.4f %10.4f %10.1f %8.4f\n", v.name.c_str(), med, v.ms[0], gbs, gbs / 8000.0);
  }
  return 0;
}
