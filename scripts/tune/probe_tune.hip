// probe_tune.hip — shapes of the write-only / read-only HBM probes behind
// gp_hbm_probe (tuning harness, not product code; it #includes the product
// kernels).  4 GiB buffer, interleaved rounds, median.  Usage: probe_tune [rounds]
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

template <int U, bool NT>
__global__ __launch_bounds__(kBlock) void wprobe(f4 *__restrict__ out, size_t n4) {
  const size_t tile = (size_t)kBlock * U;
  const size_t stride = (size_t)gridDim.x * tile;
  const f4 z = f4(0.0f);
  size_t base = (size_t)blockIdx.x * tile + threadIdx.x;
  for (; base + (U - 1) * kBlock < n4; base += stride)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT)
        __builtin_nontemporal_store(z, out + base + u * kBlock);
      else
        out[base + u * kBlock] = z;
    }
  for (int u = 0; u < U; ++u)
    if (base + u * kBlock < n4) out[base + u * kBlock] = z;
}

template <int U, bool NT>
__global__ __launch_bounds__(kBlock) void rprobe(const f4 *__restrict__ in, size_t n4, float *sink) {
  const size_t tile = (size_t)kBlock * U;
  const size_t stride = (size_t)gridDim.x * tile;
  f4 acc = f4(0.0f);
  size_t base = (size_t)blockIdx.x * tile + threadIdx.x;
  for (; base + (U - 1) * kBlock < n4; base += stride) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(in + base + u * kBlock) : in[base + u * kBlock];
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u];
  }
  if (acc.x + acc.y + acc.z + acc.w == -1234.5f) sink[blockIdx.x % 64] = acc.x;
}

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 7;
  const size_t n = (size_t)1 << 30;  // floats (4 GiB)
  float *buf;
  CK(hipMalloc(&buf, n * 4));
  CK(hipMemset(buf, 0, n * 4));
  f4 *b4 = reinterpret_cast<f4 *>(buf);
  const size_t n4 = n / 4;
  const size_t G = num_cus();
  struct V {
    std::string name;
    std::function<void()> f;
    bool read;
  };
  std::vector<V> vs;
  vs.push_back({"read  prod (U8, 4/CU)", [&] { gp_hbm_probe(GP_PROBE_READ, buf, n, 0); }, true});
  vs.push_back({"write prod (U1, 4/CU)", [&] { gp_hbm_probe(GP_PROBE_WRITE, buf, n, 0); }, false});
  for (int per : {1, 2, 4}) {
    const std::string P = " /" + std::to_string(per);
    vs.push_back({"write U4 plain" + P, [=] { hipLaunchKernelGGL((wprobe<4, false>), dim3(G * per), dim3(kBlock), 0, 0, b4, n4); }, false});
    vs.push_back({"write U8 plain" + P, [=] { hipLaunchKernelGGL((wprobe<8, false>), dim3(G * per), dim3(kBlock), 0, 0, b4, n4); }, false});
    vs.push_back({"write U16 plain" + P, [=] { hipLaunchKernelGGL((wprobe<16, false>), dim3(G * per), dim3(kBlock), 0, 0, b4, n4); }, false});
    vs.push_back({"write U2 plain" + P, [=] { hipLaunchKernelGGL((wprobe<2, false>), dim3(G * per), dim3(kBlock), 0, 0, b4, n4); }, false});
    vs.push_back({"write U4 nt" + P, [=] { hipLaunchKernelGGL((wprobe<4, true>), dim3(G * per), dim3(kBlock), 0, 0, b4, n4); }, false});
  }
  for (int per : {1, 2, 4, 8}) {
    const std::string P = " /" + std::to_string(per);
    vs.push_back({"read U4 nt" + P, [=] { hipLaunchKernelGGL((rprobe<4, true>), dim3(G * per), dim3(kBlock), 0, 0, b4, n4, buf); }, true});
    vs.push_back({"read U8 nt" + P, [=] { hipLaunchKernelGGL((rprobe<8, true>), dim3(G * per), dim3(kBlock), 0, 0, b4, n4, buf); }, true});
    vs.push_back({"read U16 nt" + P, [=] { hipLaunchKernelGGL((rprobe<16, true>), dim3(G * per), dim3(kBlock), 0, 0, b4, n4, buf); }, true});
    vs.push_back({"read U8 plain" + P, [=] { hipLaunchKernelGGL((rprobe<8, false>), dim3(G * per), dim3(kBlock), 0, 0, b4, n4, buf); }, true});
  }
  vs.push_back({"memset", [&] { CK(hipMemsetAsync(buf, 0, n * 4, 0)); }, false});
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  std::vector<std::vector<float>> ms(vs.size());
  for (auto &v : vs) v.f();
  CK(hipDeviceSynchronize());
  for (int r = 0; r < rounds; ++r)
    for (size_t i = 0; i < vs.size(); ++i) {
      CK(hipEventRecord(a, 0));
      vs[i].f();
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float t = 0;
      CK(hipEventElapsedTime(&t, a, b));
      ms[i].push_back(t);
    }
  CK(hipGetLastError());
  for (size_t i = 0; i < vs.size(); ++i) {
    auto m = ms[i];
    std::sort(m.begin(), m.end());
    const double med = m[m.size() / 2];
    std::printf("%-26s %8.4f ms %8.1f GB/s\n", vs[i].name.c_str(), med, n * 4.0 / (med * 1e-3) / 1e9);
  }
  return 0;
}
