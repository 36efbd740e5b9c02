// geeps_sum_app — drives libgeeps through the unchanged public API
// (include/geeps.hpp) the way a data-parallel app does, and checks every Read.
//
//   geeps_sum_app <process_id> <num_processes> <base_port> <rows> <clocks>
//                 <slack> <channels> <read_my_writes> [int|float] [layers]
//                 [tables] [local] [output_dir]
//
// `tables` > 1 assigns blob l to table l % tables (rows numbered per table);
// `local` = 1 adds a LocalAccess(fetch) / PostLocalAccess(keep) pair whose
// buffer must carry the previous iteration's contents into the next one;
// `output_dir` sets GeePsConfig::output_dir (GetStats appends json_stats.<pid>).
// GEEPS_TEST_JITTER_US=J in the environment: before every Read and every Clock
// the process sleeps a pseudo-random 0..J us (seeded by its id), so processes
// drift apart and refreshes, master-version switches and releases interleave
// differently from run to run.
// GEEPS_TEST_EMPTY_SETUP=1: the setup clock (clock 0) carries no updates, so
// every server's first refresh is an empty shard (all zeros).
// GEEPS_TEST_SPREAD_DEVICES=1: process p works on GPU p % device_count (one
// process per GPU, as on an 8-GPU node), selected before GeePs is created.
// GEEPS_TEST_SHUFFLE_UPDATES=1: every PreUpdate lists its blob's rows in a
// shuffled order (seeded per blob), so the update op's DoubleIndex maps op
// rows to cache rows by a permutation and libgeeps' row plan reorders it;
// =odd: only the odd blobs' (the even ones can take the direct oplog).
//
// `layers` (comma-separated row counts, summing to `rows`) switches to a
// Caffe-like op sequence: a Read per parameter blob in forward order, then per
// blob in reverse order PreUpdate / PostRead / Update, then Clock.
//
// Each process declares one table of `rows` RowData rows: Read(all rows,
// slack), PreUpdate(all rows), PostRead, Update, Clock.  Process p's delta at
// clock c for element e is a small integer (exact in fp32, so the check is
// independent of the order in which the server received the processes'
// updates).  With `float` and one process the deltas are random floats and the
// expected value is the sequential fp32 sum (bit-exact).
//
// BSP (slack 0): the Read at iteration i must equal exactly the sum of every
// process's deltas for clocks 0 .. i-1 (clock 0 is the setup clock before
// StartIterations).  SSP: it must lie between the sums through clock
// i-slack-1 and through clock i+slack (deltas are positive).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "geeps.hpp"

static float delta(int p, int c, size_t e, bool fl) {
  if (fl) {
    uint32_t x = (uint32_t)(e * 2654435761u) ^ (uint32_t)(c * 40503u + p * 977u + 12345u);
    x ^= x >> 13;
    x *= 0x5bd1e995u;
    x ^= x >> 15;
    // 1 in 64 is -0.0f: the reference's oplog turns it into +0.0f (zerofy,
    // then +=); libgeeps' direct oplog keeps it, which must not change a bit
    if ((x >> 24) % 64 == 0) return -0.0f;
    return (float)(x & 0xffffff) / 16777216.0f - 0.5f;
  }
  return (float)(1 + ((p * 7 + c * 3 + e) % 5));  // 1..5
}

// GEEPS_TEST_ASYNC_READ=<n>: each Read buffer is copied by two kernels on the
// null stream, queued right after Read and never waited for before PostRead: a
// plain copy, then one that first sleeps n x s_sleep(127) (~3.4 us each) and
// copies again.  Both read the buffer before PostRead in stream order, so the
// two copies must be identical: a direct Read's master version may not go back
// to its server (which could then rewrite it) before the app's queued device
// work on it is done.
__global__ void copy_kernel(float *dst, const float *src, size_t n, int sleeps) {
  for (int i = 0; i < sleeps; ++i) __builtin_amdgcn_s_sleep(127);
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

#define HCK(x)                                                     \
  do {                                                             \
    hipError_t e_ = (x);                                           \
    if (e_ != hipSuccess) {                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
      std::exit(3);                                                \
    }                                                              \
  } while (0)

int main(int argc, char **argv) {
  if (argc < 9) {
    std::fprintf(stderr, "usage: %s pid nproc base_port rows clocks slack channels rmw [float]\n",
                 argv[0]);
    return 2;
  }
  const int pid = std::atoi(argv[1]), P = std::atoi(argv[2]), base = std::atoi(argv[3]);
  const size_t rows = std::strtoull(argv[4], 0, 10);
  const int clocks = std::atoi(argv[5]), slack = std::atoi(argv[6]);
  const int channels = std::atoi(argv[7]), rmw = std::atoi(argv[8]);
  const bool fl = argc > 9 && std::string(argv[9]) == "float";
  std::vector<size_t> layer_rows;
  if (argc > 10) {
    std::string spec = argv[10];
    size_t pos = 0;
    while (pos < spec.size()) {
      const size_t c = spec.find(',', pos);
      layer_rows.push_back(std::strtoull(spec.substr(pos, c - pos).c_str(), 0, 10));
      if (c == std::string::npos) break;
      pos = c + 1;
    }
  } else {
    layer_rows.push_back(std::strtoull(argv[4], 0, 10));
  }
  if (fl && P != 1) {
    std::fprintf(stderr, "float mode needs one process (order-independent check otherwise)\n");
    return 2;
  }
  const size_t n = rows * ROW_DATA_SIZE;
  const int T = argc > 11 ? std::atoi(argv[11]) : 1;
  const bool use_local = argc > 12 && std::atoi(argv[12]) != 0;
  const std::string out_dir = argc > 13 ? argv[13] : "";

  if (std::getenv("GEEPS_TEST_SPREAD_DEVICES")) {
    int count = 0;
    HCK(hipGetDeviceCount(&count));
    HCK(hipSetDevice(pid % count));
  }
  GeePsConfig cfg;
  cfg.num_tables = T;
  cfg.output_dir = out_dir;
  for (int i = 0; i < P; ++i) {
    cfg.host_list.push_back("127.0.0.1");
    cfg.port_list.push_back(base + 16 * i);
  }
  cfg.num_comm_channels = channels;
  cfg.read_my_writes = rmw;
  cfg.gpu_memory_capacity = (size_t)1 << 34;
  // GEEPS_TEST_CAPACITY=<bytes>: a tight gpu_memory_capacity, so key batches
  // past it go to libgeeps' host tier (vi_decide_param_cache);
  // GEEPS_TEST_MM_LEVEL=<n>: mm_warning_level (3 refuses a host tier)
  if (const char *cap = std::getenv("GEEPS_TEST_CAPACITY")) cfg.gpu_memory_capacity = std::strtoull(cap, nullptr, 10);
  if (const char *lvl = std::getenv("GEEPS_TEST_MM_LEVEL")) cfg.mm_warning_level = std::atoi(lvl);
  if (const char *pin = std::getenv("GEEPS_TEST_PINNED")) cfg.pinned_cpu_memory = std::atoi(pin);
  GeePs *ps = new GeePs(pid, cfg);

  size_t total = 0;
  for (size_t r : layer_rows) total += r;
  if (total != rows) {
    std::fprintf(stderr, "layer rows sum to %zu, not %zu\n", total, rows);
    return 2;
  }
  const size_t L = layer_rows.size();
  std::vector<size_t> first(L), table_of(L), first_in_table(L);
  std::vector<int> h_read(L), h_pre(L), h_post(L), h_upd(L);
  std::vector<size_t> next_row(T, 0);
  for (size_t l = 0, r0 = 0; l < L; r0 += layer_rows[l], ++l) {
    first[l] = r0;  // position in the app's flat value array
    table_of[l] = l % T;
    first_in_table[l] = next_row[table_of[l]];
    next_row[table_of[l]] += layer_rows[l];
  }
  auto ids_of = [&](size_t l) {
    std::vector<size_t> ids(layer_rows[l]);
    for (size_t r = 0; r < layer_rows[l]; ++r) ids[r] = first_in_table[l] + r;
    return ids;
  };
  // upd_row[l][j]: the blob row the update op's buffer row j carries
  // ("odd": only the odd blobs, so one clock mixes in-order and shuffled ops)
  const char *shuffle_env = std::getenv("GEEPS_TEST_SHUFFLE_UPDATES");
  const bool shuffle_odd = shuffle_env && std::string(shuffle_env) == "odd";
  std::vector<std::vector<size_t>> upd_row(L);
  for (size_t l = 0; l < L; ++l) {
    upd_row[l].resize(layer_rows[l]);
    for (size_t r = 0; r < layer_rows[l]; ++r) upd_row[l][r] = r;
    const bool shuffle = shuffle_env && (!shuffle_odd || l % 2 == 1);
    uint32_t st = 0x2545f491u ^ (uint32_t)(l * 2654435761u + 17);
    for (size_t r = layer_rows[l]; shuffle && r > 1; --r) {  // Fisher-Yates
      st ^= st << 13;
      st ^= st >> 17;
      st ^= st << 5;
      std::swap(upd_row[l][r - 1], upd_row[l][st % r]);
    }
  }
  auto upd_ids_of = [&](size_t l) {
    std::vector<size_t> ids(layer_rows[l]);
    for (size_t j = 0; j < layer_rows[l]; ++j) ids[j] = first_in_table[l] + upd_row[l][j];
    return ids;
  };
  const size_t local_rows = 3;
  std::vector<size_t> local_ids(local_rows);
  for (size_t r = 0; r < local_rows; ++r) local_ids[r] = 1000 + r;
  int h_local = -1, h_local_post = -1;
  if (use_local) h_local = ps->VirtualLocalAccess(local_ids, true);
  for (size_t l = 0; l < L; ++l) h_read[l] = ps->VirtualRead(table_of[l], ids_of(l), slack);
  for (size_t l = L; l-- > 0;) {
    h_pre[l] = ps->VirtualPreUpdate(table_of[l], upd_ids_of(l));
    h_post[l] = ps->VirtualPostRead(h_read[l]);
    h_upd[l] = ps->VirtualUpdate(h_pre[l]);
  }
  if (use_local) h_local_post = ps->VirtualPostLocalAccess(h_local, true);
  ps->VirtualClock();
  ps->FinishVirtualIteration();

  std::vector<float> host(n), got(n), again;
  std::vector<RowData *> rbufs(L, nullptr);
  // GEEPS_TEST_REREAD=1: each Read buffer is read again just before its
  // PostRead and must not have changed (a direct Read's master version stays
  // pinned while refreshes arrive).
  const bool reread = std::getenv("GEEPS_TEST_REREAD") != nullptr;
  const char *async_env = std::getenv("GEEPS_TEST_ASYNC_READ");
  const bool async_read = async_env != nullptr;
  const int async_sleeps = async_read ? std::atoi(async_env) : 0;
  float *dev_got = nullptr, *dev_got2 = nullptr;
  hipStream_t fill_stream = nullptr;  // async mode: fills that do not wait for the null stream
  if (async_read) {
    HCK(hipMalloc(&dev_got, n * 4));
    HCK(hipMalloc(&dev_got2, n * 4));
    HCK(hipStreamCreateWithFlags(&fill_stream, hipStreamNonBlocking));
  }
  int bad = 0;
  // PreUpdate -> fill on the device -> [PostRead] -> Update, in declared order.
  auto push = [&](int c, bool post_read) {
    for (size_t l = L; l-- > 0;) {
      RowOpVal *buf = nullptr;
      ps->PreUpdate(h_pre[l], &buf);
      const size_t e0 = first[l] * ROW_DATA_SIZE, ne = layer_rows[l] * ROW_DATA_SIZE;
      for (size_t j = 0; j < layer_rows[l]; ++j)  // buffer row j carries blob row upd_row[l][j]
        for (size_t v = 0; v < ROW_DATA_SIZE; ++v)
          host[e0 + j * ROW_DATA_SIZE + v] =
              delta(pid, c, e0 + upd_row[l][j] * ROW_DATA_SIZE + v, fl);
      if (async_read) {
        HCK(hipMemcpyAsync(buf, host.data() + e0, ne * 4, hipMemcpyHostToDevice, fill_stream));
        HCK(hipStreamSynchronize(fill_stream));
      } else {
        HCK(hipMemcpy(buf, host.data() + e0, ne * 4, hipMemcpyHostToDevice));
      }
      if (post_read && reread && !async_read) {
        again.resize(ne);
        HCK(hipMemcpy(again.data(), rbufs[l], ne * 4, hipMemcpyDeviceToHost));
        if (std::memcmp(again.data(), got.data() + e0, ne * 4) != 0 && bad < 5) {
          std::fprintf(stderr, "p%d clock %d layer %zu: Read buffer changed before PostRead\n", pid, c, l);
          ++bad;
        }
      }
      if (post_read) ps->PostRead(h_post[l]);
      ps->Update(h_upd[l]);
    }
  };
  // Expected sums through clock k, over all processes, in the order the
  // single-process server applies them (k = -1: zeros).
  const bool empty_setup = std::getenv("GEEPS_TEST_EMPTY_SETUP") != nullptr;
  std::vector<std::vector<float>> through(clocks + 2, std::vector<float>(n, 0.0f));
  for (int k = 0; k <= clocks; ++k) {
    through[k + 1] = through[k];
    if (k == 0 && empty_setup) continue;
    for (int p = 0; p < P; ++p)
      for (size_t e = 0; e < n; ++e) through[k + 1][e] += delta(p, k, e, fl);
  }
  auto sum_through = [&](int k) -> const std::vector<float> & {
    if (k < -1) k = -1;
    if (k > clocks) k = clocks;
    return through[k + 1];
  };

  // Setup clock (clock 0) before StartIterations, as apps/helloworld does.
  if (!empty_setup) push(0, false);
  ps->Clock();
  ps->StartIterations();

  std::vector<float> lbuf(local_rows * ROW_DATA_SIZE);
  const char *jit = std::getenv("GEEPS_TEST_JITTER_US");
  const unsigned jitter_us = jit ? (unsigned)std::strtoul(jit, nullptr, 10) : 0;
  uint32_t jstate = 0x9e3779b9u ^ (uint32_t)(pid * 7919 + 1);
  auto jitter = [&] {
    if (!jitter_us) return;
    jstate ^= jstate << 13;
    jstate ^= jstate >> 17;
    jstate ^= jstate << 5;
    std::this_thread::sleep_for(std::chrono::microseconds(jstate % (jitter_us + 1)));
  };
  for (int it = 1; it <= clocks; ++it) {
    if (use_local) {
      // Local data persists across iterations: it holds what we wrote last time.
      RowData *lp = nullptr;
      ps->LocalAccess(h_local, &lp);
      HCK(hipMemcpy(lbuf.data(), lp, lbuf.size() * 4, hipMemcpyDeviceToHost));
      const float want = it == 1 ? 0.0f : (float)(pid * 100 + it - 1);
      for (size_t i = 0; i < lbuf.size() && bad < 5; ++i)
        if (lbuf[i] != want) {
          std::fprintf(stderr, "p%d it%d local %zu: got %g expected %g\n", pid, it, i, lbuf[i], want);
          ++bad;
        }
      for (auto &v : lbuf) v = (float)(pid * 100 + it);
      HCK(hipMemcpy(lp, lbuf.data(), lbuf.size() * 4, hipMemcpyHostToDevice));
    }
    for (size_t l = 0; l < L; ++l) {
      RowData *rbuf = nullptr;
      jitter();
      ps->Read(h_read[l], &rbuf);
      rbufs[l] = rbuf;
      const size_t e0 = first[l] * ROW_DATA_SIZE, ne = layer_rows[l] * ROW_DATA_SIZE;
      if (async_read) {
        const float *src = reinterpret_cast<const float *>(rbuf);
        hipLaunchKernelGGL(copy_kernel, dim3(64), dim3(256), 0, 0, dev_got + e0, src, ne, 0);
        hipLaunchKernelGGL(copy_kernel, dim3(64), dim3(256), 0, 0, dev_got2 + e0, src, ne, async_sleeps);
        HCK(hipGetLastError());
      } else {
        HCK(hipMemcpy(got.data() + e0, rbuf, ne * 4, hipMemcpyDeviceToHost));
      }
    }
    if (async_read) {
      // PostRead (inside push) while the copies may still run; then both copies
      // of every buffer must agree
      push(it, true);
      HCK(hipDeviceSynchronize());
      again.resize(n);
      HCK(hipMemcpy(got.data(), dev_got, n * 4, hipMemcpyDeviceToHost));
      HCK(hipMemcpy(again.data(), dev_got2, n * 4, hipMemcpyDeviceToHost));
      for (size_t l = 0; l < L && bad < 5; ++l) {
        const size_t e0 = first[l] * ROW_DATA_SIZE, ne = layer_rows[l] * ROW_DATA_SIZE;
        if (std::memcmp(again.data() + e0, got.data() + e0, ne * 4) != 0) {
          std::fprintf(stderr, "p%d it%d layer %zu: Read buffer changed under device work queued "
                       "before PostRead\n", pid, it, l);
          ++bad;
        }
      }
    }
    if (slack == 0 && !rmw) {
      const auto &e = sum_through(it - 1);
      for (size_t i = 0; i < n && bad < 5; ++i) {
        if (std::memcmp(&got[i], &e[i], 4) != 0) {
          std::fprintf(stderr, "p%d it%d elem %zu: got %.9g expected %.9g\n", pid, it, i, got[i], e[i]);
          ++bad;
        }
      }
    } else if (!fl) {
      const auto &lo = sum_through(it - slack - 1);
      const auto &hi = sum_through(it + slack + (rmw ? 1 : 0));
      for (size_t i = 0; i < n && bad < 5; ++i) {
        if (!(got[i] >= lo[i] && got[i] <= hi[i])) {
          std::fprintf(stderr, "p%d it%d elem %zu: got %g outside [%g, %g]\n", pid, it, i, got[i],
                       lo[i], hi[i]);
          ++bad;
        }
      }
    }
    if (!async_read) push(it, true);
    if (use_local) ps->PostLocalAccess(h_local_post);
    jitter();
    ps->Clock();
  }
  std::string stats = ps->GetStats();
  std::printf("%s p%d rows=%zu layers=%zu tables=%d local=%d clocks=%d slack=%d channels=%d rmw=%d %s\n",
              bad ? "MISMATCH" : "OK", pid, rows, L, T, (int)use_local, clocks, slack, channels,
              rmw, fl ? "float" : "int");
  std::printf("stats %s\n", stats.c_str());
  std::fflush(stdout);
  ps->Shutdown();
  return bad ? 1 : 0;
}
