#ifndef GEEPS_AMD_NET_HPP_
#define GEEPS_AMD_NET_HPP_

// Socket ends of the reduction path.  The reference moves update pushes and
// shard refreshes over ZeroMQ ROUTER sockets (src/common/router-handler.cpp);
// libgeeps uses plain TCP with a minimal multipart framing whose PARTS are the
// reference's message frames byte for byte (wire.hpp):
//
//   frame := magic u32 'GPS1' | nparts u32 | len u64 x nparts | part bytes ...
//
// A connection opens with one HELLO frame carrying the client's process id.
// Only the framing differs from ZMQ's ZMTP; the payloads decode with the
// reference's structs unchanged.

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace geeps {

constexpr uint32_t kFrameMagic = 0x31535047u;  // "GPS1"
constexpr uint32_t kHelloCmd = 0x48454c4fu;    // "HELO"

// First frame on a client -> server connection.
struct HelloMsg {
  uint32_t cmd;         // kHelloCmd
  uint32_t process_id;  // the connecting client
  uint32_t ipc;         // it takes same-node refreshes in place
  uint32_t pad;
  char pci_bus_id[32];  // its GPU (gp_device_pci_bus_id): a peer on another GPU
                        // has its IPC-mapped buckets copied to local HBM first
};

struct Part {
  const void *data;
  size_t size;
};

// Blocking helpers on a connected socket.  Return false on EOF / error.
bool send_frame(int fd, const std::vector<Part> &parts);
// Reads one frame; `alloc(i, size)` returns where part i goes (nullptr = a
// temporary vector owned by `scratch`).
struct RecvPart {
  void *data;
  size_t size;
};
bool recv_frame(int fd, std::vector<RecvPart> &parts,
                std::vector<std::vector<char>> &scratch,
                void *(*alloc)(void *ctx, size_t index, size_t size), void *ctx);

int listen_tcp(uint16_t port, std::string *err);
int accept_tcp(int listen_fd);
// Connect with retries until `timeout_s` elapses.
int connect_tcp(const std::string &host, uint16_t port, double timeout_s, std::string *err);
void close_fd(int fd);
void shutdown_fd(int fd);

}  // namespace geeps

#endif  // GEEPS_AMD_NET_HPP_
