#ifndef GEEPS_AMD_CLIENT_INTERNAL_HPP_
#define GEEPS_AMD_CLIENT_INTERNAL_HPP_

// Helpers shared by ClientLib's translation units (client.cpp, client_viter.cpp,
// client_data.cpp, client_net.cpp): not part of libgeeps' interface.

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <memory>
#include <string>
#include <vector>

#include "client.hpp"

namespace geeps {
namespace client_detail {

inline double now_s() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

constexpr size_t kRowBytes = sizeof(RowData);
// How long a client retries connecting to a server that is not listening yet
// (processes start at different times); GEEPS_CONNECT_TIMEOUT_S overrides.
inline double connect_timeout_s() {
  const char *e = std::getenv("GEEPS_CONNECT_TIMEOUT_S");
  const double v = e ? std::atof(e) : 0.0;
  return v > 0 ? v : 300.0;
}
constexpr int kWaitWarnMs = 12000;  // the reference's 12 s timed_wait warnings

// GEEPS_IPC_LOG=1: one stderr line per IPC handle exported or mapped (which
// buffer, where, how large), on both sides, to audit buffer lifetimes.
inline bool ipc_log() {
  static const bool on = std::getenv("GEEPS_IPC_LOG") != nullptr;
  return on;
}

// gp_ipc_describe_handle's line on an exported handle (the exporter's pid,
// base and size; the process and address the runtime's handle names), for
// the GEEPS_IPC_LOG lines: a run's log then pairs every mapping with the
// export it came from.
inline std::string ipc_describe(const void *handle) {
  char buf[400];
  if (gp_ipc_describe_handle(handle, buf, sizeof buf) != GP_OK) return std::string("(") + gp_last_error() + ")";
  return buf;
}

// A reader thread's pinned receive buffers: one is reused once no batch holds
// it.  use_count() is a relaxed load; the acquire fence after it pairs with the
// release in the last holder's decrement (another thread: the server, done
// with the rows), so this thread's next writes follow that holder's use.
struct PinnedPool {
  std::vector<std::shared_ptr<PinnedArray<float>>> bufs;
  std::shared_ptr<PinnedArray<float>> get(size_t floats) {
    for (auto &b : bufs)
      if (b.use_count() == 1 && b->size() >= floats) {
        std::atomic_thread_fence(std::memory_order_acquire);
        return b;
      }
    bufs.push_back(std::make_shared<PinnedArray<float>>(std::max<size_t>(floats, 1)));
    return bufs.back();
  }
};

// Rows bound for a socket leave the GPU in pieces of this size, each sent as
// soon as its copy lands (send_frame_chunked), so the D2H of a large slice
// overlaps the send instead of preceding it.
constexpr size_t kWireChunk = 16u << 20;

// The device-to-host copy of `bytes` from `src` into pinned `dst` on `st`, an
// event recorded after each kWireChunk piece.
inline void copy_out_in_pieces(void *dst, const void *src, size_t bytes, const Stream &st,
                        std::vector<std::unique_ptr<Event>> &events) {
  const size_t pieces = (bytes + kWireChunk - 1) / kWireChunk;
  while (events.size() < pieces) events.push_back(std::make_unique<Event>());
  for (size_t k = 0; k < pieces; ++k) {
    const size_t off = k * kWireChunk, len = std::min(kWireChunk, bytes - off);
    GP_CALL(gp_memcpy_async(static_cast<char *>(dst) + off, static_cast<const char *>(src) + off, len, st.get()));
    events[k]->record(st);
  }
}

}  // namespace client_detail
}  // namespace geeps

#endif  // GEEPS_AMD_CLIENT_INTERNAL_HPP_
