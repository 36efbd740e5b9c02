/*
 * oracle.c — CPU restatement of the GeePS gradient-update reduction path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (geeps_amd/, the C-ABI
 * library, libgeeps) links, loads or calls this file.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg use it — as the
 * checker and as the reported CPU baseline, never as the thing measured.
 *
 * Parity status: the reference's own arithmetic (math_functions.cpp,
 * row-op-util.hpp) cannot be compiled in this image without writing stand-ins
 * for glog / cblas / zmq.hpp / CUDA headers, which this project does not do,
 * and the reference ships no tests or golden vectors.  The ARITHMETIC of this
 * restatement is therefore "parity unpinned" against the reference binary; it
 * is pinned only by re-statement (each function cites the lines it follows)
 * and by hand-computed known answers in tests/test_oracle.py.  The DATA
 * LAYOUT it assumes (RowData = 128 floats, DoubleIndex / RowKey = 16 B, wire
 * headers) IS pinned against the reference's own headers, compiled unchanged
 * by oracle/Makefile into oracle/_ref/layout_probe.
 *
 * Built by oracle/Makefile with `gcc -O3` and no -march, matching the
 * reference's CCFLAGS (SConscript:34-38: -O3, no arch flags).
 */
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

/* vsAdd: y[i] = a[i] + b[i]
 * src/common/gpu-util/mkl_alternate.hpp:59-74 (DEFINE_VSL_BINARY_FUNC(Add)),
 * reached through cpu_add<float> (src/common/gpu-util/math_functions.cpp:132-136).
 * The reference takes `int n` and CHECK_GT(n, 0)s (aborts); this restatement
 * takes a 64-bit count and returns -1 where the reference would abort. */
int oracle_vs_add(int64_t n, const float *a, const float *b, float *y) {
  if (n <= 0 || !a || !b || !y) return -1;
  for (int64_t i = 0; i < n; ++i) y[i] = a[i] + b[i];
  return 0;
}

/* add_rows_from_double_index_cpu — src/common/row-op-util.hpp:121-139.
 * `index` holds num_rows {id0, id1} pairs (DoubleIndex, :40-44). */
void oracle_add_rows_from_double_index(float *y, const float *x,
                                       const uint64_t *index, size_t num_rows,
                                       uint64_t off0, uint64_t off1,
                                       size_t row_size, size_t num_vals_limit) {
  for (size_t r = 0; r < num_rows; ++r) {
    const size_t row_from = index[2 * r] + off0;     /* id0 */
    const size_t row_to = index[2 * r + 1] + off1;   /* id1 */
    for (size_t v = 0; v < row_size; ++v) {
      const size_t x_idx = row_from * row_size + v;
      const size_t y_idx = row_to * row_size + v;
      if (x_idx < num_vals_limit) y[y_idx] += x[x_idx];
    }
  }
}

/* assign_rows_to_double_index_cpu — src/common/row-op-util.hpp:81-99. */
void oracle_assign_rows_to_double_index(float *y, const float *x,
                                        const uint64_t *index, size_t num_rows,
                                        uint64_t off0, uint64_t off1,
                                        size_t row_size, size_t num_vals_limit) {
  for (size_t r = 0; r < num_rows; ++r) {
    const size_t row_from = index[2 * r + 1] + off1; /* id1 */
    const size_t row_to = index[2 * r] + off0;       /* id0 */
    for (size_t v = 0; v < row_size; ++v) {
      const size_t x_idx = row_from * row_size + v;
      const size_t y_idx = row_to * row_size + v;
      if (y_idx < num_vals_limit) y[y_idx] = x[x_idx];
    }
  }
}

/* assign_rows_from_double_index_cpu — src/common/row-op-util.hpp:101-119. */
void oracle_assign_rows_from_double_index(float *y, const float *x,
                                          const uint64_t *index,
                                          size_t num_rows, uint64_t off0,
                                          uint64_t off1, size_t row_size,
                                          size_t num_vals_limit) {
  for (size_t r = 0; r < num_rows; ++r) {
    const size_t row_from = index[2 * r] + off0;     /* id0 */
    const size_t row_to = index[2 * r + 1] + off1;   /* id1 */
    for (size_t v = 0; v < row_size; ++v) {
      const size_t x_idx = row_from * row_size + v;
      const size_t y_idx = row_to * row_size + v;
      if (x_idx < num_vals_limit) y[y_idx] = x[x_idx];
    }
  }
}

/* The server's N-way sum: TabletStorage::apply_updates
 * (src/server/tablet-server.cpp:119-134) runs once per client message, each
 * time cpu_add(num_vals, master, update, master); messages are applied in
 * arrival order, modelled here as updates[0..n_clients-1]. */
int oracle_apply_updates(float *master, const float *const *updates,
                         int n_clients, int64_t num_vals) {
  for (int c = 0; c < n_clients; ++c) {
    const int rc = oracle_vs_add(num_vals, master, updates[c], master);
    if (rc) return rc;
  }
  return 0;
}

/* Row-range partition of a param cache over servers
 * (src/client/clientlib-viter.cpp:674-682). */
void oracle_server_partition(size_t num_rows, size_t num_servers,
                             uint64_t *row_start, uint64_t *num_rows_out) {
  const size_t div = num_rows / num_servers;
  const size_t res = num_rows % num_servers;
  for (size_t i = 0; i < num_servers; ++i) {
    row_start[i] = div * i + (res > i ? i : res);
    num_rows_out[i] = div + (res > i ? 1 : 0);
  }
}

/* Multi-channel form of oracle_apply_updates for the CPU baseline: the
 * reference runs one tablet-server thread per communication channel
 * (src/client/clientlib.cpp:102-105) and splits rows over channels by
 * contiguous range (src/client/clientlib.cpp:216-224); each channel's server
 * thread applies the client messages for ITS rows in arrival order.  Same
 * per-element arithmetic and order as oracle_apply_updates. */
typedef struct {
  float *master;
  const float *const *updates;
  int n_clients;
  int64_t begin, end;
} oracle_chunk;

static void *oracle_chunk_run(void *arg) {
  oracle_chunk *c = (oracle_chunk *)arg;
  for (int k = 0; k < c->n_clients; ++k) {
    if (c->end > c->begin)
      oracle_vs_add(c->end - c->begin, c->master + c->begin,
                    c->updates[k] + c->begin, c->master + c->begin);
  }
  return NULL;
}

int oracle_apply_updates_mt(float *master, const float *const *updates,
                            int n_clients, int64_t num_vals, int threads) {
  enum { kMaxThreads = 256 };
  if (threads < 1) threads = 1;
  if (threads > kMaxThreads) threads = kMaxThreads;
  if (threads == 1) return oracle_apply_updates(master, updates, n_clients, num_vals);
  pthread_t tid[kMaxThreads];
  oracle_chunk chunk[kMaxThreads];
  const int64_t div = num_vals / threads, res = num_vals % threads;
  for (int t = 0; t < threads; ++t) {
    const int64_t b = div * t + (res > t ? t : res);
    chunk[t].master = master;
    chunk[t].updates = updates;
    chunk[t].n_clients = n_clients;
    chunk[t].begin = b;
    chunk[t].end = b + div + (res > t ? 1 : 0);
    if (pthread_create(&tid[t], NULL, oracle_chunk_run, &chunk[t]) != 0) return -2;
  }
  for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
  return 0;
}

/* Synthetic deltas for the CPU baseline at full table size (bench.py): fp32
 * uniform in [-0.5, 0.5) from a per-(seed, block) splitmix64 stream, filled
 * by `threads` threads.  Not the reference's arithmetic (it has no data
 * generator); only the timed oracle_apply_updates* above is. */
typedef struct {
  float *p;
  int64_t begin, end;
  uint64_t seed;
} oracle_fill_job;

static uint64_t oracle_splitmix(uint64_t *s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static void *oracle_fill_run(void *arg) {
  oracle_fill_job *j = (oracle_fill_job *)arg;
  uint64_t s = j->seed ^ ((uint64_t)j->begin * 0xD1B54A32D192ED03ull);
  for (int64_t i = j->begin; i < j->end; ++i)
    j->p[i] = (float)(oracle_splitmix(&s) >> 40) * (1.0f / 16777216.0f) - 0.5f;
  return NULL;
}

int oracle_fill_uniform(float *p, int64_t n, uint64_t seed, int threads) {
  enum { kMaxThreads = 256 };
  if (threads < 1) threads = 1;
  if (threads > kMaxThreads) threads = kMaxThreads;
  pthread_t tid[kMaxThreads];
  oracle_fill_job job[kMaxThreads];
  const int64_t div = n / threads, res = n % threads;
  for (int t = 0; t < threads; ++t) {
    const int64_t b = div * t + (res > t ? t : res);
    job[t].p = p;
    job[t].begin = b;
    job[t].end = b + div + (res > t ? 1 : 0);
    job[t].seed = seed;
    if (pthread_create(&tid[t], NULL, oracle_fill_run, &job[t]) != 0) return -2;
  }
  for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
  return 0;
}
