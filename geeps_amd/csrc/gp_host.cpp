// Host-memory row ops of the C-ABI (include/gp_reduce.h, ABI 13-15): the
// reference's CPU twins of the row ops (src/common/row-op-util.hpp:64-139),
// which libgeeps' host tier runs on the rows a param cache keeps in host
// memory past `gpu_memory_capacity` (src/client/clientlib-viter.cpp:492-611).
//
// Each loop visits the index entries in order, as the reference's does, so a
// destination listed twice gets its adds in op order.  Two changes of shape,
// neither of which changes a bit of the result:
//   * a whole row under the limit runs as a straight, vectorisable loop, and
//     only the row that straddles `num_vals_limit` is guarded per element;
//   * a large call runs on several threads, each owning a contiguous range of
//     DESTINATION rows and walking the whole index in order for the entries
//     that land there: every destination still gets its entries in index
//     order, from one thread (the reference's loop is one thread; a host tier
//     of a large table is memory-bound, and one core reads ~10 GB/s).
//     Threads: GP_HOST_THREADS, else OMP_NUM_THREADS, else the hardware's,
//     at most 32; calls under 4 MiB of rows stay on the calling thread.  The
//     helper threads are a persistent pool (a host tier calls these several
//     times a clock, and starting 15 threads per call cost more than the
//     copies it overlaps).
#include <pthread.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <system_error>
#include <thread>
#include <unordered_set>
#include <utility>
#include <vector>

#include "gp_reduce.h"

namespace gp_internal {
int set_error(int code, const char *msg);  // gp_reduce.hip: the thread's gp_last_error
}  // namespace gp_internal

namespace {

// Rows past num_vals_limit on the guarded side contribute nothing; a row is
// whole when its last element is under the limit.  (val_id, row_size and
// the products are 64-bit: the reference's size_t.)
template <typename F>
inline void guarded_row(size_t base, size_t row_size, size_t limit, F &&f) {
  if (base + row_size <= limit) {
    for (size_t v = 0; v < row_size; ++v) f(v);
  } else if (base < limit) {
    for (size_t v = 0; v < limit - base; ++v) f(v);
  }
}

int host_error(const char *msg) { return gp_internal::set_error(GP_ERR_INVALID, msg); }

unsigned host_threads() {
  static const unsigned n = [] {
    for (const char *name : {"GP_HOST_THREADS", "OMP_NUM_THREADS"})
      if (const char *e = std::getenv(name)) {
        const long v = std::strtol(e, nullptr, 10);
        if (v > 0) return (unsigned)std::min<long>(v, 32);
      }
    const unsigned hw = std::thread::hardware_concurrency();
    return std::max(1u, std::min(hw, 32u));
  }();
  return n;
}

constexpr size_t kParallelBytes = 4u << 20;

// Worker threads shared by every caller (the app thread and libgeeps' reader
// threads call these concurrently).  A call queues its tasks 1 .. t-1, runs
// task 0, then runs any of its own tasks no worker has taken yet, and waits
// for the rest.  Workers start on first need and are never joined (the
// process's exit ends them); a forked child starts a pool of its own.
class Pool {
 public:
  static Pool &get() {
    static std::once_flag once;
    std::call_once(once, [] { pthread_atfork(nullptr, nullptr, [] { instance().store(nullptr); }); });
    Pool *p = instance().load(std::memory_order_acquire);
    if (p) return *p;
    Pool *mine = new Pool();  // (leaked on purpose, see above)
    if (instance().compare_exchange_strong(p, mine, std::memory_order_acq_rel)) return *mine;
    delete mine;  // another thread's came first
    return *p;
  }

  void run(unsigned t, const std::function<void(unsigned)> &task) {
    Call c;
    c.task = &task;
    c.left = t - 1;
    {
      std::lock_guard<std::mutex> lk(mu_);
      try {
        while (workers_ < t - 1) {
          std::thread([this] { work(); }).detach();
          ++workers_;
        }
      } catch (const std::system_error &) {
        // (no more threads: the caller runs the tasks no worker takes)
      }
      for (unsigned k = 1; k < t; ++k) q_.emplace_back(&c, k);
    }
    cv_.notify_all();
    task(0);
    for (;;) {  // this call's tasks still queued
      unsigned k = 0;
      {
        std::lock_guard<std::mutex> lk(mu_);
        auto it = std::find_if(q_.begin(), q_.end(), [&](const std::pair<Call *, unsigned> &e) { return e.first == &c; });
        if (it == q_.end()) break;
        k = it->second;
        q_.erase(it);
      }
      task(k);
      finish(&c);
    }
    std::unique_lock<std::mutex> lk(c.mu);
    c.cv.wait(lk, [&] { return c.left == 0; });
  }

 private:
  struct Call {
    const std::function<void(unsigned)> *task = nullptr;
    unsigned left = 0;  // under mu
    std::mutex mu;
    std::condition_variable cv;
  };
  static std::atomic<Pool *> &instance() {
    static std::atomic<Pool *> p{nullptr};
    return p;
  }
  // (under c->mu to the end: the caller may return as soon as it sees 0)
  static void finish(Call *c) {
    std::lock_guard<std::mutex> lk(c->mu);
    if (--c->left == 0) c->cv.notify_one();
  }
  void work() {
    for (;;) {
      std::pair<Call *, unsigned> e;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return !q_.empty(); });
        e = q_.front();
        q_.pop_front();
      }
      (*e.first->task)(e.second);
      finish(e.first);
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::pair<Call *, unsigned>> q_;
  unsigned workers_ = 0;
};

// Runs body(lo, hi) over [0, n) split into contiguous ranges, one per thread
// (the calling thread takes the first).
template <typename F>
void parallel_ranges(size_t n, size_t bytes, F &&body) {
  const unsigned t = bytes < kParallelBytes ? 1u : (unsigned)std::min<size_t>(host_threads(), n);
  if (t <= 1) {
    body((size_t)0, n);
    return;
  }
  const size_t per = (n + t - 1) / t;
  Pool::get().run(t, [&](unsigned k) {
    const size_t lo = std::min(n, k * per), hi = std::min(n, lo + per);
    if (lo < hi) body(lo, hi);
  });
}

// The destination rows an index writes, [lo, hi) (offsets applied), for the
// destination-range split.
template <bool TO_ID1>
void dest_span(const gp_double_index *index, size_t n, gp_double_index off, size_t *lo, size_t *hi) {
  size_t a = SIZE_MAX, b = 0;
  for (size_t i = 0; i < n; ++i) {
    const size_t d = (TO_ID1 ? index[i].id1 + off.id1 : index[i].id0 + off.id0);
    a = std::min(a, d);
    b = std::max(b, d);
  }
  *lo = a;
  *hi = b + 1;
}

}  // namespace

extern "C" {

int gp_host_scatter_add_rows(float *y, const float *x, const gp_double_index *index, size_t num_rows,
                             gp_double_index offset, size_t row_size, size_t num_vals_limit) {
  if (num_rows == 0) return GP_OK;
  if (!y || !x || !index || row_size == 0) return host_error("gp_host_scatter_add_rows: bad argument");
  size_t d0 = 0, d1 = 0;
  const size_t bytes = num_rows * row_size * sizeof(float);
  if (bytes >= kParallelBytes) dest_span<true>(index, num_rows, offset, &d0, &d1);
  parallel_ranges(d1 - d0, bytes, [&](size_t lo, size_t hi) {
    const bool all = bytes < kParallelBytes;  // one thread: every entry
    for (size_t i = 0; i < num_rows; ++i) {
      const size_t from = index[i].id0 + offset.id0, to = index[i].id1 + offset.id1;
      if (!all && (to < d0 + lo || to >= d0 + hi)) continue;
      const float *__restrict__ xs = x + from * row_size;
      float *__restrict__ ys = y + to * row_size;
      // the guard is on the source (x) index, row-op-util.hpp:133-135
      guarded_row(from * row_size, row_size, num_vals_limit, [&](size_t v) { ys[v] += xs[v]; });
    }
  });
  return GP_OK;
}

int gp_host_scatter_init_rows(float *y, const float *x, const gp_double_index *index, size_t num_rows,
                              gp_double_index offset, size_t row_size, size_t num_vals_limit) {
  if (num_rows == 0) return GP_OK;
  if (!y || !x || !index || row_size == 0) return host_error("gp_host_scatter_init_rows: bad argument");
  size_t d0 = 0, d1 = 0;
  const size_t bytes = num_rows * row_size * sizeof(float);
  dest_span<true>(index, num_rows, offset, &d0, &d1);
  parallel_ranges(d1 - d0, bytes, [&](size_t lo, size_t hi) {
    // a destination's first entry initialises it (0.0f + x, 0.0f past the
    // limit: the zerofied row plus its add), any later one adds, in entry
    // order: zerofy + add for any index, repeated destinations included
    const bool dense = hi - lo <= 8 * num_rows + 1024;
    std::vector<uint8_t> seen(dense ? hi - lo : 0, 0);
    std::unordered_set<size_t> seen_sparse;
    for (size_t i = 0; i < num_rows; ++i) {
      const size_t from = index[i].id0 + offset.id0, to = index[i].id1 + offset.id1;
      if (to < d0 + lo || to >= d0 + hi) continue;
      bool first;
      if (dense) {
        uint8_t &s = seen[to - d0 - lo];
        first = !s;
        s = 1;
      } else {
        first = seen_sparse.insert(to).second;
      }
      const float *__restrict__ xs = x + from * row_size;
      float *__restrict__ ys = y + to * row_size;
      const size_t base = from * row_size;
      if (!first) {
        guarded_row(base, row_size, num_vals_limit, [&](size_t v) { ys[v] += xs[v]; });
      } else if (base + row_size <= num_vals_limit) {
        for (size_t v = 0; v < row_size; ++v) ys[v] = 0.0f + xs[v];
      } else {
        for (size_t v = 0; v < row_size; ++v) ys[v] = base + v < num_vals_limit ? 0.0f + xs[v] : 0.0f;
      }
    }
  });
  return GP_OK;
}

int gp_host_gather_rows(float *y, const float *x, const gp_double_index *index, size_t num_rows,
                        gp_double_index offset, size_t row_size, size_t num_vals_limit) {
  if (num_rows == 0) return GP_OK;
  if (!y || !x || !index || row_size == 0) return host_error("gp_host_gather_rows: bad argument");
  size_t d0 = 0, d1 = 0;
  const size_t bytes = num_rows * row_size * sizeof(float);
  if (bytes >= kParallelBytes) dest_span<false>(index, num_rows, offset, &d0, &d1);
  parallel_ranges(d1 - d0, bytes, [&](size_t lo, size_t hi) {
    const bool all = bytes < kParallelBytes;
    for (size_t i = 0; i < num_rows; ++i) {
      const size_t from = index[i].id1 + offset.id1, to = index[i].id0 + offset.id0;
      if (!all && (to < d0 + lo || to >= d0 + hi)) continue;
      const float *__restrict__ xs = x + from * row_size;
      float *__restrict__ ys = y + to * row_size;
      // the guard is on the destination (y, the op buffer) index, row-op-util.hpp:93-95
      guarded_row(to * row_size, row_size, num_vals_limit, [&](size_t v) { ys[v] = xs[v]; });
    }
  });
  return GP_OK;
}

int gp_host_add(size_t n, float *y, const float *x) {
  if (n == 0) return GP_OK;
  if (!y || !x) return host_error("gp_host_add: null pointer");
  parallel_ranges(n, n * sizeof(float), [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) y[i] += x[i];
  });
  return GP_OK;
}

int gp_host_zero(size_t n, float *y) {
  if (n == 0) return GP_OK;
  if (!y) return host_error("gp_host_zero: null pointer");
  parallel_ranges(n, n * sizeof(float), [&](size_t lo, size_t hi) {
    std::memset(y + lo, 0, (hi - lo) * sizeof(float));
  });
  return GP_OK;
}

}  // extern "C"
