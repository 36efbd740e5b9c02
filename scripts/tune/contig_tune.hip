// contig_tune.hip — does a physically contiguous allocation make the 8-way
// sweep sum's rate independent of where the allocation lands (tuning harness,
// not product code; it #includes the product kernels)?  Over fresh
// allocations after random spacers the production 8-way sum ran 80.7-87.2 %
// of 8 TB/s (profiles/r02/tune/sum_alloc2.txt); the bench's arena, the
// process's first large allocation, sits at the top.  Each round here
// allocates a spacer of random size, then the 36-GiB arena (8 buckets +
// master) once with hipMalloc and once with hipExtMallocWithFlags(...,
// hipDeviceMallocContiguous), times gp_bucket_sum_apply over each (5 calls,
// median, HIP events) and frees both.  Results are bit-checked between the two.
// Usage: contig_tune [rounds]
#include "../../geeps_amd/csrc/gp_reduce.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
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

__global__ void fill_k(float *p, size_t n, unsigned seed) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    unsigned v = (unsigned)(i * 2654435761u) ^ seed;
    v ^= v >> 13;
    v *= 0x5bd1e995u;
    v ^= v >> 15;
    p[i] = (float)(v & 0xffffff) / 16777216.0f - 0.5f;
  }
}

__global__ void diff_k(const unsigned *a, const unsigned *b, size_t n, unsigned long long *bad) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  unsigned long long c = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) c += a[i] != b[i];
  if (c) atomicAdd(bad, c);
}

// fills the arena, runs the 8-way sum 1 + 5 times, returns the median ms
float time_arena(char *a) {
  const size_t stride = kN * 4;
  const float *bk[8];
  for (int k = 0; k < 8; ++k) {
    fill_k<<<4096, 256>>>(reinterpret_cast<float *>(a + (size_t)k * stride), kN, 1000 + k);
    bk[k] = reinterpret_cast<const float *>(a + (size_t)k * stride);
  }
  float *m = reinterpret_cast<float *>(a + (size_t)8 * stride);
  fill_k<<<4096, 256>>>(m, kN, 77);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> ms;
  for (int r = 0; r < 6; ++r) {
    CK(hipEventRecord(e0, 0));
    if (gp_bucket_sum_apply(m, bk, 8, kN, nullptr) != GP_OK) std::exit(3);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float t = 0;
    CK(hipEventElapsedTime(&t, e0, e1));
    if (r) ms.push_back(t);
  }
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  std::sort(ms.begin(), ms.end());
  return ms[ms.size() / 2];
}

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 6;
  const size_t bytes = 9 * kN * 4;
  const double algo = 10.0 * kN * 4;  // (8 + 2) streams
  std::mt19937 rng(5);
  unsigned long long *bad = nullptr;
  CK(hipMalloc(&bad, 8));
  std::printf("round spacer_MiB  default ms      %%  contiguous ms      %%  mismatches\n");
  std::vector<void *> spacers;
  for (int r = 0; r < rounds; ++r) {
    const size_t sp = (size_t)(rng() % 4096 + 1) << 20;
    void *s = nullptr;
    CK(hipMalloc(&s, sp));
    spacers.push_back(s);
    char *a = nullptr, *c = nullptr;
    CK(hipMalloc(reinterpret_cast<void **>(&a), bytes));
    const float ta = time_arena(a);
    const hipError_t ec = hipExtMallocWithFlags(reinterpret_cast<void **>(&c), bytes, hipDeviceMallocContiguous);
    if (ec != hipSuccess) {
      std::printf("%5d %10zu  %10.4f %6.2f  contiguous allocation failed: %s\n", r, sp >> 20, ta,
                  100.0 * algo / (ta * 1e-3) / 8e12, hipGetErrorString(ec));
      (void)hipGetLastError();
      CK(hipFree(a));
      continue;
    }
    const float tc = time_arena(c);
    CK(hipMemset(bad, 0, 8));
    diff_k<<<4096, 256>>>(reinterpret_cast<const unsigned *>(a + 8 * kN * 4),
                          reinterpret_cast<const unsigned *>(c + 8 * kN * 4), kN, bad);
    unsigned long long hb = 0;
    CK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
    std::printf("%5d %10zu  %10.4f %6.2f  %13.4f %6.2f  %llu\n", r, sp >> 20, ta, 100.0 * algo / (ta * 1e-3) / 8e12,
                tc, 100.0 * algo / (tc * 1e-3) / 8e12, hb);
    CK(hipFree(a));
    CK(hipFree(c));
  }
  for (void *s : spacers) CK(hipFree(s));
  return 0;
}
