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

int main(int argc, char **argv) {
  if (argc < 7) {
    std::fprintf(stderr, "usage: %s pid nproc base_port rows clocks warmup\n", argv[0]);
    return 2;
  }
  const int pid = std::atoi(argv[1]), P = std::atoi(argv[2]), base = std::atoi(argv[3]);
  const size_t rows = std::strtoull(argv[4], 0, 10);
  const int clocks = std::atoi(argv[5]), warmup = std::atoi(argv[6]);
  const int slack = argc > 7 ? std::atoi(argv[7]) : 0;
  GeePsConfig cfg;
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
  for (int s = 0; s < (per_shard ? P : 1); ++s) {
    const size_t div = rows / P, res = rows % P;
    const size_t lo = per_shard ? div * s + std::min<size_t>(s, res) : 0;
    const size_t hi = per_shard ? lo + div + ((size_t)s < res ? 1 : 0) : rows;
    hr.push_back(ps->VirtualRead(0, std::vector<size_t>(ids.begin() + lo, ids.begin() + hi), slack));
  }
  const int hp = ps->VirtualPreUpdate(0, ids);
  for (int h : hr) hpr.push_back(ps->VirtualPostRead(h));
  const int hu = ps->VirtualUpdate(hp);
  ps->VirtualClock();
  ps->FinishVirtualIteration();

  RowOpVal *ub = nullptr;
  ps->PreUpdate(hp, &ub);
  HCK(hipMemset(ub, 0, rows * sizeof(RowOpVal)));
  ps->Update(hu);
  ps->Clock();
  ps->StartIterations();

  using clk = std::chrono::steady_clock;
  clk::time_point t0;
  for (int c = 0; c < warmup + clocks; ++c) {
    if (c == warmup) t0 = clk::now();
    RowData *rb = nullptr;
    for (int h : hr) ps->Read(h, &rb);
    ps->PreUpdate(hp, &ub);
    // the app's "gradient": 0.5 everywhere, written on the device
    HCK(hipMemsetD32(reinterpret_cast<hipDeviceptr_t>(ub), 0x3f000000, rows * ROW_DATA_SIZE));
    HCK(hipDeviceSynchronize());
    for (int h : hpr) ps->PostRead(h);
    ps->Update(hu);
    ps->Clock();
  }
  // the last Read waits for the last clock's refresh: include it
  RowData *rb = nullptr;
  for (int h : hr) ps->Read(h, &rb);
  const double s = std::chrono::duration<double>(clk::now() - t0).count();
  float probe = 0;
  HCK(hipMemcpy(&probe, rb, 4, hipMemcpyDeviceToHost));
  const double per = s / clocks;
  const double table_bytes = (double)rows * sizeof(RowData);
  std::printf("{\"process\": %d, \"processes\": %d, \"rows\": %zu, \"table_bytes\": %.0f, "
              "\"slack\": %d, \"clocks\": %d, \"ms_per_clock\": %.4f, \"delta_GBps\": %.2f, \"probe\": %.1f}\n",
              pid, P, rows, table_bytes, slack, clocks, per * 1e3, table_bytes / per / 1e9, probe);
  std::fflush(stdout);
  std::fprintf(stderr, "stats %s\n", ps->GetStats().c_str());
  ps->Shutdown();
  return 0;
}
