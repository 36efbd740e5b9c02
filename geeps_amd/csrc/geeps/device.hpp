#ifndef GEEPS_AMD_DEVICE_HPP_
#define GEEPS_AMD_DEVICE_HPP_

// RAII owners for device memory, pinned host memory, streams and events, all
// through the C-ABI (include/gp_reduce.h) so that no HIP type appears in the
// host library.

#include <cstddef>
#include <iostream>
#include <memory>
#include <string>
#include <utility>

#include "check.hpp"
#include "gp_reduce.h"
#include "hostshare.hpp"

namespace geeps {

// Page-locked host memory through the C-ABI.  In a ThreadSanitizer build
// (scripts/build_tsan.sh) the HIP runtime's allocator is not instrumented:
// TSan cannot see that a block one thread freed and another thread got back
// from the runtime was ordered by the runtime's own locking, and reports the
// two threads' accesses to it as a race.  The free releases and the
// allocation acquires on the block's address, stating that edge.
#if defined(__has_feature)
#if __has_feature(thread_sanitizer)
extern "C" void __tsan_acquire(void *addr);
extern "C" void __tsan_release(void *addr);
#define GEEPS_TSAN_ACQUIRE(p) __tsan_acquire(p)
#define GEEPS_TSAN_RELEASE(p) __tsan_release(p)
#endif
#endif
#ifndef GEEPS_TSAN_ACQUIRE
#define GEEPS_TSAN_ACQUIRE(p) ((void)(p))
#define GEEPS_TSAN_RELEASE(p) ((void)(p))
#endif

inline void *pinned_alloc(size_t bytes) {
  void *p = nullptr;
  GP_CALL(gp_malloc_host(&p, bytes));
  GEEPS_TSAN_ACQUIRE(p);
  return p;
}

inline int pinned_free(void *p) {
  GEEPS_TSAN_RELEASE(p);
  return gp_free_host(p);
}

class Stream {
 public:
  Stream() { GP_CALL(gp_stream_create(&s_)); }
  ~Stream() {
    if (s_) gp_stream_destroy(s_);
  }
  Stream(const Stream &) = delete;
  Stream &operator=(const Stream &) = delete;
  gp_stream get() const { return s_; }
  void sync() const { GP_CALL(gp_stream_synchronize(s_)); }

 private:
  gp_stream s_ = nullptr;
};

class Event {
 public:
  Event() { GP_CALL(gp_event_create(&e_)); }
  ~Event() {
    if (e_) gp_event_destroy(e_);
  }
  Event(const Event &) = delete;
  Event &operator=(const Event &) = delete;
  void record(const Stream &s) { GP_CALL(gp_event_record(e_, s.get())); }
  // the legacy default (null) stream: where an app's own device work goes
  void record_default() { GP_CALL(gp_event_record(e_, nullptr)); }
  void sync() { GP_CALL(gp_event_synchronize(e_)); }
  gp_event get() const { return e_; }

 private:
  gp_event e_ = nullptr;
};

// A device (HBM) array of T.  `shared`: a buffer peers map over IPC (oplogs,
// master versions), allocated whole (gp_malloc_device_shared: >= 2 MiB, never a
// fragment of a block the runtime sub-allocates).
struct SharedAlloc {};
constexpr SharedAlloc kShared{};

template <typename T>
class DeviceArray {
 public:
  DeviceArray() = default;
  explicit DeviceArray(size_t n) { resize(n); }
  DeviceArray(size_t n, SharedAlloc) : shared_(true) { resize(n); }
  ~DeviceArray() { release(); }
  DeviceArray(const DeviceArray &) = delete;
  DeviceArray &operator=(const DeviceArray &) = delete;
  DeviceArray(DeviceArray &&o) noexcept { swap(o); }
  DeviceArray &operator=(DeviceArray &&o) noexcept {
    if (this != &o) {
      release();
      swap(o);
    }
    return *this;
  }
  void resize(size_t n) {
    release();
    if (n) {
      void *p = nullptr;
      if (shared_)
        GP_CALL(gp_malloc_device_shared(&p, n * sizeof(T)));
      else
        GP_CALL(gp_malloc_device(&p, n * sizeof(T)));
      p_ = static_cast<T *>(p);
    }
    n_ = n;
  }
  void release() {
    if (p_) GP_CALL(gp_free_device(p_));
    p_ = nullptr;
    n_ = 0;
  }
  void swap(DeviceArray &o) noexcept {
    std::swap(p_, o.p_);
    std::swap(n_, o.n_);
    std::swap(shared_, o.shared_);
  }
  T *data() const { return p_; }
  size_t size() const { return n_; }
  size_t bytes() const { return n_ * sizeof(T); }

 private:
  T *p_ = nullptr;
  size_t n_ = 0;
  bool shared_ = false;
};

// Page-locked host memory (the reference's mallocHost, common-util.hpp).
template <typename T>
class PinnedArray {
 public:
  PinnedArray() = default;
  explicit PinnedArray(size_t n) { resize(n); }
  ~PinnedArray() { release(); }
  PinnedArray(const PinnedArray &) = delete;
  PinnedArray &operator=(const PinnedArray &) = delete;
  void resize(size_t n) {
    release();
    if (n) p_ = static_cast<T *>(pinned_alloc(n * sizeof(T)));
    n_ = n;
  }
  void release() {
    if (p_) GP_CALL(pinned_free(p_));
    p_ = nullptr;
    n_ = 0;
  }
  T *data() const { return p_; }
  size_t size() const { return n_; }

 private:
  T *p_ = nullptr;
  size_t n_ = 0;
};

// Host memory of libgeeps' host tier (the rows a param cache keeps in CPU
// memory past gpu_memory_capacity): page-locked when `pinned` (the config's
// pinned_cpu_memory, default on), so its copies to and from HBM run at the
// pinned PCIe rate; plain memory otherwise, as the reference's DataStorage::CPU.
// `shareable` (pinned host oplogs with a same-node server): shared memory a
// peer can map (hostshare.hpp), private pinned memory if the system refuses it.
class HostBuf {
 public:
  HostBuf(size_t n, bool pinned, bool shareable = false) : n_(n), pinned_(pinned) {
    if (!n) return;
    if (pinned && shareable) {
      std::string why;
      shm_ = SharedHostMem::create(n * sizeof(float), &why);
      if (shm_) {
        p_ = static_cast<float *>(shm_->data());
        return;
      }
      std::cerr << "libgeeps: shared host memory refused (" << why
                << "); this host oplog's rows go to same-node servers by socket\n";
    }
    if (pinned) {
      p_ = static_cast<float *>(pinned_alloc(n * sizeof(float)));
    } else {
      p_ = new float[n];
    }
  }
  ~HostBuf() {
    if (!p_ || shm_) return;  // (shm_ unmaps itself)
    if (pinned_)
      pinned_free(p_);
    else
      delete[] p_;
  }
  HostBuf(const HostBuf &) = delete;
  HostBuf &operator=(const HostBuf &) = delete;
  float *data() const { return p_; }
  size_t size() const { return n_; }
  void zero() { GP_CALL(gp_host_zero(n_, p_)); }  // zerofy_data_cpu, threaded when large
  const SharedHostMem *shared() const { return shm_.get(); }  // null: private memory

 private:
  std::unique_ptr<SharedHostMem> shm_;
  float *p_ = nullptr;
  size_t n_ = 0;
  bool pinned_ = false;
};

// A row plan: a DoubleIndex compiled once, on the current device, for the ops
// whose index is fixed after FinishVirtualIteration -- a scatter plan
// (gp_row_plan_create) for Update, a gather plan (gp_gather_plan_create) for
// Read.
class RowPlan {
 public:
  RowPlan(const gp_double_index *host_index, size_t n, size_t row_size, size_t num_vals_limit,
          bool gather = false) {
    if (gather)
      GP_CALL(gp_gather_plan_create(&p_, host_index, n, gp_double_index{0, 0}, row_size, num_vals_limit));
    else
      GP_CALL(gp_row_plan_create(&p_, host_index, n, gp_double_index{0, 0}, row_size, num_vals_limit));
  }
  ~RowPlan() {
    if (p_) gp_row_plan_destroy(p_);
  }
  RowPlan(const RowPlan &) = delete;
  RowPlan &operator=(const RowPlan &) = delete;
  gp_row_plan get() const { return p_; }

 private:
  gp_row_plan p_ = nullptr;
};

}  // namespace geeps

#endif  // GEEPS_AMD_DEVICE_HPP_
