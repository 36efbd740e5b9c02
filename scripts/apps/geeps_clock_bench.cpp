// geeps_clock_bench — end-to-end clock rate of libgeeps through the public API.
//
//   geeps_clock_bench <process_id> <num_processes> <base_port> <rows> <clocks> <warmup> [slack]
//
// One table of `rows` RowData rows; per clock the app does what apps/helloworld
// does, at scale: Read(all rows) -> PreUpdate(all rows) -> PostRead -> Update
// -> Clock, with the update buffer filled on the device.  A clock therefore runs
// the whole reduction path: oplog zero + row-indexed scatter-add (Update), the
// push of each server's slice (zero-copy in process, D2H + TCP otherwise), the
// server's bucket sum into its master shard, the refresh of every client's
// param cache, and the gather into the Read buffer.  Prints one JSON line.
// CLOCK_BENCH_READ_PER_SHARD=1 declares one Read op per server shard instead
// (as per-blob ops mostly fall within one shard), which direct reads
// (GEEPS_DIRECT_READ=1) can hand out in place.
// GEEPS_TEST_SPREAD_DEVICES=1: process p works on GPU p % device_count (one
// process per GPU, as on an 8-GPU node), selected before GeePs is created.
//
// Read check: every worker adds 0.5 to every element each clock (the setup
// clock adds 0), so the last Read after K timed + warm-up clocks must hold
// 0.5 * P * K in every element at slack 0 (exact in fp32), and lie in
// [0.5 * P * (K - slack), 0.5 * P * K] under SSP.  A device kernel counts the
// elements outside that range over every Read buffer ("read_bad").
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "geeps.hpp"

#define HCK(x)                                                     \
  do {                                                             \
    hipError_t e_ = (x);                                           \
    if (e_ != hipSuccess) {                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
      std::exit(3);                                                \
    }                                                              \
  } while (0)

__global__ void count_outside(const float *x, size_t n, float lo, float hi, unsigned long long *bad) {
  unsigned long long local = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float v = x[i];
    local += (v >= lo && v <= hi) ? 0 : 1;
  }
  if (local) atomicAdd(bad, local);
}

int main(int argc, char **argv) {
  if (argc < 7) {
    std::fprintf(stderr, "usage: %s pid nproc base_port rows clocks warmup\n", argv[0]);
    return 2;
  }
  const int pid = std::atoi(argv[1]), P = std::atoi(argv[2]), base = std::atoi(argv[3]);
  const size_t rows = std::strtoull(argv[4], 0, 10);
  const int clocks = std::atoi(argv[5]), warmup = std::atoi(argv[6]);
  const int slack = argc > 7 ? std::atoi(argv[7]) : 0;
  int device = 0;
  if (std::getenv("GEEPS_TEST_SPREAD_DEVICES")) {
    int count = 0;
    HCK(hipGetDeviceCount(&count));
    device = pid % count;
  }
  HCK(hipSetDevice(device));
  GeePsConfig cfg;
  // CLOCK_BENCH_RMW: read-my-writes (each Read adds this worker's own
  // unpushed updates to the refreshed rows, clientlib-data.cpp:132-150)
  if (std::getenv("CLOCK_BENCH_RMW")) cfg.read_my_writes = 1;
  // CLOCK_BENCH_HOST_TIER_FRAC=f: the table's rows as two key batches (rows
  // [0, h) and [h, rows), h = (1 - f) rows), each read and updated by an op of
  // its own, and a gpu_memory_capacity that holds the thread cache (twice the
  // peak rows in use: both Reads and both PreUpdates, 2 x rows) and the first
  // batch only (2 rows of capacity per cached row: the cache and one oplog),
  // so the second batch, f of the rows, lives in libgeeps' host tier
  // (vi_decide_param_cache, clientlib-viter.cpp:520-568)
  const char *frac_env = std::getenv("CLOCK_BENCH_HOST_TIER_FRAC");
  const double host_frac = frac_env ? std::atof(frac_env) : 0.0;
  const size_t split_at = host_frac > 0 ? (size_t)((1.0 - host_frac) * (double)rows) : rows;
  if (host_frac > 0) cfg.gpu_memory_capacity = (4 * rows + 2 * split_at) * sizeof(RowData);
  for (int i = 0; i < P; ++i) {
    cfg.host_list.push_back("127.0.0.1");
    cfg.port_list.push_back(base + 16 * i);
  }
  GeePs *ps = new GeePs(pid, cfg);
  std::vector<size_t> ids(rows);
  for (size_t r = 0; r < rows; ++r) ids[r] = r;
  // the reference partition of the table's rows over the servers
  // (clientlib-viter.cpp:674-682): P contiguous ranges
  const bool per_shard = std::getenv("CLOCK_BENCH_READ_PER_SHARD") != nullptr;
  std::vector<int> hr, hpr;
  std::vector<size_t> hr_rows;
  std::vector<std::pair<size_t, size_t>> batches;  // [lo, hi) of each Read op
  if (host_frac > 0) {
    batches = {{0, split_at}, {split_at, rows}};
  } else {
    for (int s = 0; s < (per_shard ? P : 1); ++s) {
      const size_t div = rows / P, res = rows % P;
      const size_t lo = per_shard ? div * s + std::min<size_t>(s, res) : 0;
      batches.emplace_back(lo, per_shard ? lo + div + ((size_t)s < res ? 1 : 0) : rows);
    }
  }
  for (auto &b : batches) {
    hr.push_back(ps->VirtualRead(0, std::vector<size_t>(ids.begin() + b.first, ids.begin() + b.second), slack));
    hr_rows.push_back(b.second - b.first);
  }
  // one update op over the table, or one per batch (a host-tier batch is
  // updated by ops of its own)
  std::vector<std::pair<size_t, size_t>> ubatches = host_frac > 0 ? batches : std::vector<std::pair<size_t, size_t>>{{0, rows}};
  std::vector<int> hps, hus;
  for (auto &b : ubatches)
    hps.push_back(ps->VirtualPreUpdate(0, std::vector<size_t>(ids.begin() + b.first, ids.begin() + b.second)));
  for (int h : hr) hpr.push_back(ps->VirtualPostRead(h));
  for (int h : hps) hus.push_back(ps->VirtualUpdate(h));
  ps->VirtualClock();
  ps->FinishVirtualIteration();

  RowOpVal *ub = nullptr;
  for (size_t i = 0; i < hps.size(); ++i) {
    ps->PreUpdate(hps[i], &ub);
    HCK(hipMemset(ub, 0, (ubatches[i].second - ubatches[i].first) * sizeof(RowOpVal)));
  }
  for (int h : hus) ps->Update(h);
  ps->Clock();
  ps->StartIterations();

  using clk = std::chrono::steady_clock;
  clk::time_point t0;
  for (int c = 0; c < warmup + clocks; ++c) {
    if (c == warmup) t0 = clk::now();
    RowData *rb = nullptr;
    for (int h : hr) ps->Read(h, &rb);
    for (size_t i = 0; i < hps.size(); ++i) {
      ps->PreUpdate(hps[i], &ub);
      // the app's "gradient": 0.5 everywhere, written on the device
      HCK(hipMemsetD32(reinterpret_cast<hipDeviceptr_t>(ub), 0x3f000000,
                       (ubatches[i].second - ubatches[i].first) * ROW_DATA_SIZE));
    }
    HCK(hipDeviceSynchronize());
    for (int h : hpr) ps->PostRead(h);
    for (int h : hus) ps->Update(h);
    ps->Clock();
  }
  // the last Read waits for the last clock's refresh: include it
  std::vector<RowData *> last(hr.size(), nullptr);
  for (size_t i = 0; i < hr.size(); ++i) ps->Read(hr[i], &last[i]);
  const double s = std::chrono::duration<double>(clk::now() - t0).count();
  float probe = 0;
  HCK(hipMemcpy(&probe, last.back(), 4, hipMemcpyDeviceToHost));
  // every element of every Read buffer against the expected range (untimed)
  const int K = warmup + clocks;
  const float hi = 0.5f * (float)P * (float)K, lo = 0.5f * (float)P * (float)(K - slack);
  unsigned long long *dbad = nullptr, bad = 0;
  HCK(hipMalloc(&dbad, sizeof *dbad));
  HCK(hipMemset(dbad, 0, sizeof *dbad));
  size_t checked = 0;
  for (size_t i = 0; i < hr.size(); ++i) {
    const size_t n = hr_rows[i] * ROW_DATA_SIZE;
    hipLaunchKernelGGL(count_outside, dim3(1024), dim3(256), 0, 0, reinterpret_cast<const float *>(last[i]), n,
                       lo, hi, dbad);
    HCK(hipGetLastError());
    checked += n;
  }
  HCK(hipMemcpy(&bad, dbad, sizeof bad, hipMemcpyDeviceToHost));
  HCK(hipFree(dbad));
  const double per = s / clocks;
  const double table_bytes = (double)rows * sizeof(RowData);
  std::printf("{\"process\": %d, \"processes\": %d, \"device\": %d, \"rows\": %zu, \"table_bytes\": %.0f, "
              "\"slack\": %d, \"clocks\": %d, \"ms_per_clock\": %.4f, \"delta_GBps\": %.2f, \"probe\": %.1f, "
              "\"read_checked\": %zu, \"read_bad\": %llu, \"read_lo\": %.1f, \"read_hi\": %.1f}\n",
              pid, P, device, rows, table_bytes, slack, clocks, per * 1e3, table_bytes / per / 1e9, probe,
              checked, bad, lo, hi);
  std::fflush(stdout);
  std::fprintf(stderr, "stats %s\n", ps->GetStats().c_str());
  ps->Shutdown();
  return 0;
}
