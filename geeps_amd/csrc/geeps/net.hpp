#ifndef GEEPS_AMD_NET_HPP_
#define GEEPS_AMD_NET_HPP_

// Socket ends of the reduction path.  The reference moves update pushes and
// shard refreshes between ZeroMQ ROUTER sockets (src/common/router-handler.cpp:
// 69-120): each client's ROUTER ("client-<i>") connects to every server's
// ROUTER ("tablet-<i>", bound on tcp_base_port + channel, server-entry.cpp:
// 56-68), and one message is a multipart of the reference's structs
// (encoder-decoder.cpp:105-150, server-encoder-decoder.cpp:228-250).
//
// libgeeps speaks the same wire protocol natively, with no ZeroMQ library:
// ZMTP/3.0 with the NULL security mechanism as a ROUTER socket.
//
//   greeting  0xFF 0*8 0x7F | version 3.0 | "NULL" + 0*16 | as-server 0 | 0*31
//   READY     command frame: "READY" + properties Socket-Type=ROUTER,
//             Identity=client-<i> | tablet-<i>, plus libgeeps' own X-Geeps-*
//             properties (same-node IPC, the GPU's PCI bus id)
//   message   frames: flags (0x01 MORE, 0x02 LONG) | size u8 or u64 BE | body
//
// One TCP connection per (client, server) pair carries both directions, as the
// reference's ROUTER-to-ROUTER connection does.  A stock libzmq ROUTER peer
// interoperates (tests/test_zmtp.py drives one through ctypes).

#include <cstddef>
#include <cstdint>
#include <functional>
#include <string>
#include <utility>
#include <vector>

namespace geeps {

struct Part {
  const void *data;
  size_t size;
};

// A ZMTP peer as its READY command described it.
struct PeerInfo {
  std::string socket_type;
  std::string identity;
  std::vector<std::pair<std::string, std::string>> props;  // every property, in order
  const std::string *prop(const std::string &name) const;   // case-insensitive
};

// ZMTP/3.0 NULL handshake on a connected socket: greeting both ways, then our
// READY (Socket-Type ROUTER, Identity `identity`, then `extra`) and the peer's.
// False with `*err` set on EOF, a non-ZMTP-3 peer, another mechanism, an ERROR
// command, a socket type a ROUTER cannot talk to, or a peer silent for
// `timeout_s` (a ZMTP/1.0 peer, libzmq 2.x, is refused as "not a ZMTP 2+
// endpoint").
bool zmtp_handshake(int fd, const std::string &identity,
                    const std::vector<std::pair<std::string, std::string>> &extra, PeerInfo *peer,
                    std::string *err, double timeout_s = 60.0);

// One multipart message (every part but the last flagged MORE).  Blocking.
bool send_frame(int fd, const std::vector<Part> &parts);
// The same message, its last part written in `chunk`-byte pieces, piece k
// once `ready(k)` returns (its device-to-host copy has landed): the socket
// carries the first pieces while later ones still come off the GPU.  The
// bytes on the wire are send_frame's.
bool send_frame_chunked(int fd, const std::vector<Part> &parts, size_t chunk,
                        const std::function<void(size_t)> &ready);
// Reads one multipart message; `alloc(i, size)` returns where part i goes
// (nullptr = a temporary vector owned by `scratch`).  Command frames between
// messages (PING, PONG, ...) are skipped, and a PING is not answered (the
// reference never turns on ZeroMQ heartbeats); an ERROR command ends the
// connection.  False on EOF / error / more than kMaxParts parts.
struct RecvPart {
  void *data;
  size_t size;
};
constexpr size_t kMaxParts = 64;
bool recv_frame(int fd, std::vector<RecvPart> &parts,
                std::vector<std::vector<char>> &scratch,
                void *(*alloc)(void *ctx, size_t index, size_t size), void *ctx);
// The same, reading each part in `chunk`-byte pieces and calling
// `landed(index, offset, length)` as each piece is in place (the refresh's
// host-to-device copy follows the socket piece by piece).
bool recv_frame_chunked(int fd, std::vector<RecvPart> &parts, std::vector<std::vector<char>> &scratch,
                        void *(*alloc)(void *ctx, size_t index, size_t size), void *ctx, size_t chunk,
                        const std::function<void(size_t, size_t, size_t)> &landed);

int listen_tcp(uint16_t port, std::string *err);
int accept_tcp(int listen_fd);
// Connect with retries until `timeout_s` elapses.
int connect_tcp(const std::string &host, uint16_t port, double timeout_s, std::string *err);
void close_fd(int fd);
void shutdown_fd(int fd);

}  // namespace geeps

#endif  // GEEPS_AMD_NET_HPP_
