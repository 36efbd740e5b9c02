// bucket_policy_tune.hip — cache-policy probe for the N-way bucket sum
// (tuning harness, not product code).  The production kernel's loop shape
// (U = 4 block-strides per thread, 2 blocks per CU), with every load and store
// issued as a buffer op whose `aux` cache bits are set per variant
// (gfx950: sc0 = 1, nt = 2, sc1 = 16).  The descriptors are rebuilt per block
// tile from wave-uniform values (16-KiB records), so the offsets stay 32-bit.
// One arena, buckets then master (the production layout).  Interleaved rounds
// in ONE process, median per variant.  Usage: bucket_policy_tune [rounds]
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

constexpr int kU = 4;
constexpr int kNB = 8;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, bytes, 0x00020000);
}

template <int AUX_B, int AUX_M, int AUX_S>
__global__ __launch_bounds__(kBlock) void bsum_buf(float *__restrict__ master, BucketPtrs b,
                                                   size_t n4) {
  const size_t tile = (size_t)kBlock * kU;  // f4 per block tile
  const size_t ntiles = n4 / tile;         // full tiles only (the harness size is a multiple)
  const uint32_t tbytes = (uint32_t)(tile * 16);
  const uint32_t voff = threadIdx.x * 16;
  for (size_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const size_t byte0 = t * tile * 16;
    const __amdgpu_buffer_rsrc_t rm = rsrc(reinterpret_cast<char *>(master) + byte0, tbytes);
    f4 acc[kU];
    f4 v[kNB][kU];
#pragma unroll
    for (int u = 0; u < kU; ++u)
      acc[u] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rm, voff + u * kBlock * 16, 0, AUX_M));
#pragma unroll
    for (int k = 0; k < kNB; ++k) {
      const __amdgpu_buffer_rsrc_t rb = rsrc(reinterpret_cast<const char *>(b.p[k]) + byte0, tbytes);
#pragma unroll
      for (int u = 0; u < kU; ++u)
        v[k][u] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rb, voff + u * kBlock * 16, 0, AUX_B));
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
#pragma unroll
      for (int k = 0; k < kNB; ++k) acc[u] += v[k][u];
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, acc[u]),
                                             rm, voff + u * kBlock * 16, 0, AUX_S);
    }
  }
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
  const size_t n = (1ull << 20) * 1024, n4 = n / 4;
  char *ar = nullptr;
  CK(hipMalloc(&ar, 9 * n * 4));
  BucketPtrs B{};
  for (int k = 0; k < kNB; ++k) {
    B.p[k] = reinterpret_cast<const float *>(ar + (size_t)k * n * 4);
    fill_k<<<4096, 256>>>(reinterpret_cast<float *>(ar + (size_t)k * n * 4), n, 1000 + k);
  }
  float *m = reinterpret_cast<float *>(ar + (size_t)8 * n * 4);
  fill_k<<<4096, 256>>>(m, n, 77);
  CK(hipDeviceSynchronize());
  const unsigned grid = (unsigned)num_cus() * 2;
  const double bytes = 10.0 * n * 4;

  struct V {
    std::string name;
    std::function<void()> run;
    std::vector<float> ms;
  };
  std::vector<V> vs;
#define ADD(NAME, ...) vs.push_back(V{NAME, [=]() { __VA_ARGS__; }, {}})
  const float *bk[8];
  for (int k = 0; k < 8; ++k) bk[k] = B.p[k];
  ADD("prod (global, nt buckets)", (gp_bucket_sum_apply(m, bk, 8, n, nullptr)));
  ADD("buf B=nt   M=0  S=0", (bsum_buf<2, 0, 0><<<grid, kBlock>>>(m, B, n4)));
  ADD("buf B=0    M=0  S=0", (bsum_buf<0, 0, 0><<<grid, kBlock>>>(m, B, n4)));
  ADD("buf B=sc1  M=0  S=0", (bsum_buf<16, 0, 0><<<grid, kBlock>>>(m, B, n4)));
  ADD("buf B=sc01 M=0  S=0", (bsum_buf<17, 0, 0><<<grid, kBlock>>>(m, B, n4)));
  ADD("buf B=nt1  M=0  S=0", (bsum_buf<18, 0, 0><<<grid, kBlock>>>(m, B, n4)));
  ADD("buf B=nt01 M=0  S=0", (bsum_buf<19, 0, 0><<<grid, kBlock>>>(m, B, n4)));
  ADD("buf B=nt   M=nt S=0", (bsum_buf<2, 2, 0><<<grid, kBlock>>>(m, B, n4)));
  ADD("buf B=nt   M=0  S=nt", (bsum_buf<2, 0, 2><<<grid, kBlock>>>(m, B, n4)));
  ADD("buf B=nt   M=nt S=nt", (bsum_buf<2, 2, 2><<<grid, kBlock>>>(m, B, n4)));
  ADD("buf B=nt   M=0  S=sc1", (bsum_buf<2, 0, 16><<<grid, kBlock>>>(m, B, n4)));
  ADD("buf B=nt01 M=nt01 S=nt01", (bsum_buf<19, 19, 19><<<grid, kBlock>>>(m, B, n4)));

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
    std::fprintf(stderr, "round %d done\n", r);
  }
  std::printf("%-28s %10s %10s %10s %8s\n", "variant", "med_ms", "min_ms", "GB/s", "frac8T");
  for (auto &v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const double med = v.ms[v.ms.size() / 2];
    const double gbs = bytes / (med * 1e-3) / 1e9;
    std::printf("%-28s %10.4f %10.4f %10.1f %8.4f\n", v.name.c_str(), med, v.ms[0], gbs, gbs / 8000.0);
  }
  return 0;
}
