#ifndef GEEPS_AMD_HOSTSHARE_HPP_
#define GEEPS_AMD_HOSTSHARE_HPP_

// Host memory shared with same-node peer processes (round 5): the host tier's
// oplogs.  A same-node server stages a client's host-tier rows into its bucket
// straight from the client's oplog, as it reads the HBM tier's rows through an
// IPC mapping, instead of receiving them through the socket.
//
// The buffer is a memfd mapping (no name under /dev/shm to leak), page-locked
// in every process that maps it (gp_host_register) so that its copies to HBM
// run at the pinned PCIe rate.  A peer opens it through /proc/<pid>/fd/<fd>.
// A peer maps only a descriptor that names one of these memfds, whose size is
// the handle's, and whose last page holds the handle's 16-byte tag (random per
// buffer): the descriptor number could name other memory by then, as an IPC
// handle can (gp_ipc_open_handle's tag).

#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>

namespace geeps {

struct HostShareHandle {
  int32_t pid = 0;
  int32_t fd = -1;
  uint64_t map_bytes = 0;  // the whole mapping: the rows, then the tag page
  uint8_t tag[16] = {};
};

class SharedHostMem {
 public:
  // `bytes` of zero-filled shared memory; null, with the reason in *why, when
  // the system refuses it (the caller then uses private pinned memory).
  static std::unique_ptr<SharedHostMem> create(size_t bytes, std::string *why);
  // A peer's buffer; null, with the reason in *why, when it cannot be opened
  // or mapped, or does not hold the handle's tag.
  static std::unique_ptr<SharedHostMem> open(const HostShareHandle &h, std::string *why);
  ~SharedHostMem();
  SharedHostMem(const SharedHostMem &) = delete;
  SharedHostMem &operator=(const SharedHostMem &) = delete;

  void *data() const { return base_; }
  size_t bytes() const { return bytes_; }          // usable bytes (before the tag page)
  bool pinned() const { return registered_; }      // page-locked in this process
  const HostShareHandle &handle() const { return h_; }  // what a peer opens it by

 private:
  SharedHostMem() = default;
  void *base_ = nullptr;
  size_t bytes_ = 0, map_bytes_ = 0;
  int fd_ = -1;  // the owner keeps its descriptor open for the peers
  bool registered_ = false;
  HostShareHandle h_{};
};

}  // namespace geeps

#endif  // GEEPS_AMD_HOSTSHARE_HPP_
