// r3_camp_tune.hip — round-3 probe 9 (tuning harness, not product code; it
// #includes the product kernels): why the wave-map kernel runs an IDENTITY
// index slower than a random one ("init ident wave" 59.6 % vs
// "init sorted wave" 76.1 % in profiles/r03/tune/r3_row_tune.txt).
// Hypothesis: with an identity index every wave reads row i of x and writes
// row i of y at the same moment; when x and y sit at the same offset modulo
// the HBM channel interleave, each read and its write land on the same
// channel (and bank), so the streams collide.  A random index spreads the
// reads over every channel.  Test: the production row_wave_kernel (fused init
// and gather) on an identity index with y's base moved by `shift` bytes
// relative to x's alignment, 0 B .. 2 MiB; if the hypothesis holds, some
// shifts recover the random-index rate.
// Usage: r3_camp_tune [rounds]
#include "../../geeps_amd/csrc/gp_reduce.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <numeric>
#include <random>
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

constexpr size_t R = 8u << 20, W = 128, N = R * W;
constexpr size_t kPad = 4u << 20;  // bytes of slack after y for the shifts

template <int OP>
void launch_wave(float *y, const float *x, const gp_double_index *ix, size_t n) {
  auto *kern = &row_wave_kernel<f4, OP, 32, 8, kFlat, 0>;
  static std::atomic<int> occ{0};
  const size_t grid = (size_t)num_cus() * resident_blocks(reinterpret_cast<const void *>(kern), occ);
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(kBlock), 0, 0, y, x, ix, n, 0, 0, W, W / 4, ~size_t(0),
                     SegArg<kFlat>{});
}

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 5;
  std::mt19937_64 g(9);
  std::vector<gp_double_index> ident(R), rnd(R);
  std::vector<uint64_t> perm(R);
  std::iota(perm.begin(), perm.end(), 0);
  std::shuffle(perm.begin(), perm.end(), g);
  for (size_t r = 0; r < R; ++r) {
    ident[r] = {r, r};
    rnd[r] = {perm[r], r};  // init: y[r] = 0 + x[perm[r]], destination-sorted
  }
  gp_double_index *iid, *irnd;
  CK(hipMalloc(&iid, R * 16));
  CK(hipMalloc(&irnd, R * 16));
  CK(hipMemcpy(iid, ident.data(), R * 16, hipMemcpyHostToDevice));
  CK(hipMemcpy(irnd, rnd.data(), R * 16, hipMemcpyHostToDevice));
  float *x, *ybase;
  CK(hipMalloc(&x, N * 4));
  CK(hipMalloc(&ybase, N * 4 + kPad));
  {
    std::vector<float> h(N);
    std::uniform_real_distribution<float> d(-0.5f, 0.5f);
    for (size_t i = 0; i < N; ++i) h[i] = d(g);
    CK(hipMemcpy(x, h.data(), N * 4, hipMemcpyHostToDevice));
  }
  std::printf("x %% 2 MiB = %zu, y %% 2 MiB = %zu\n", (size_t)((uintptr_t)x % (2u << 20)),
              (size_t)((uintptr_t)ybase % (2u << 20)));
  struct V {
    std::string name;
    std::function<void()> f;
  };
  std::vector<V> vs;
  const size_t shifts[] = {0, 256, 512, 1024, 2048, 4096, 8192, 16384, 65536, 262144, 1u << 20, 2u << 20};
  for (size_t sh : shifts) {
    float *y = ybase + sh / 4;
    vs.push_back({"init  ident  y shift " + std::to_string(sh), [=] { launch_wave<kInitFrom>(y, x, iid, R); }});
  }
  for (size_t sh : {(size_t)0, (size_t)4096, (size_t)(1u << 20)}) {
    float *y = ybase + sh / 4;
    vs.push_back({"gath  ident  y shift " + std::to_string(sh), [=] { launch_wave<kAssignTo>(y, x, iid, R); }});
    vs.push_back({"init  random y shift " + std::to_string(sh), [=] { launch_wave<kInitFrom>(y, x, irnd, R); }});
  }
  // the copy the dense plan uses, for scale
  vs.push_back({"dense sweep ZIN (plan path)", [&] {
                  BucketPtrs b = {};
                  b.p[0] = x;
                  launch_bucket_sum_nb<1, true>(ybase, nullptr, b, N, 0);
                }});
  // check one shift against the unshifted result
  {
    float *y0 = ybase, *y1 = ybase + 4096 / 4;
    launch_wave<kInitFrom>(y0, x, iid, R);
    CK(hipDeviceSynchronize());
    std::vector<float> a(4096), b(4096);
    CK(hipMemcpy(a.data(), y0 + (N / 2), 4096 * 4, hipMemcpyDeviceToHost));
    launch_wave<kInitFrom>(y1, x, iid, R);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(b.data(), y1 + (N / 2), 4096 * 4, hipMemcpyDeviceToHost));
    for (int i = 0; i < 4096; ++i)
      if (std::memcmp(&a[i], &b[i], 4)) {
        std::printf("check: shifted result differs at %d\n", i);
        return 3;
      }
  }
  hipEvent_t ea, eb;
  CK(hipEventCreate(&ea));
  CK(hipEventCreate(&eb));
  std::vector<std::vector<float>> ms(vs.size());
  for (auto &v : vs) v.f();
  CK(hipDeviceSynchronize());
  for (int r = 0; r < rounds; ++r)
    for (size_t i = 0; i < vs.size(); ++i) {
      CK(hipEventRecord(ea, 0));
      vs[i].f();
      CK(hipEventRecord(eb, 0));
      CK(hipEventSynchronize(eb));
      float t = 0;
      CK(hipEventElapsedTime(&t, ea, eb));
      ms[i].push_back(t);
    }
  CK(hipGetLastError());
  std::printf("8M rows x 512 B; bytes = 2 x rows + 16 B index per row\n");
  std::printf("%-32s %9s %9s %8s\n", "variant", "med_ms", "min_ms", "%8TB/s");
  const double bytes = 2.0 * N * 4 + 16.0 * R;
  for (size_t i = 0; i < vs.size(); ++i) {
    auto m = ms[i];
    std::sort(m.begin(), m.end());
    const double med = m[m.size() / 2];
    std::printf("%-32s %9.4f %9.4f %7.1f%%\n", vs[i].name.c_str(), med, m[0], 100.0 * bytes / (med * 1e-3) / 8e12);
  }
  return 0;
}
