// ZMTP/3.0 ROUTER transport for libgeeps — see net.hpp.
#include "net.hpp"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <sys/uio.h>
#include <unistd.h>

#include <endian.h>
#include <limits.h>

#include <algorithm>
#include <cctype>
#include <cerrno>
#include <chrono>
#include <cstring>
#include <thread>

namespace geeps {

namespace {

bool write_all(int fd, const void *p, size_t n) {
  const char *c = static_cast<const char *>(p);
  while (n) {
    const ssize_t w = ::send(fd, c, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    c += w;
    n -= (size_t)w;
  }
  return true;
}

bool read_all(int fd, void *p, size_t n) {
  char *c = static_cast<char *>(p);
  while (n) {
    const ssize_t r = ::recv(fd, c, n, 0);
    if (r == 0) return false;
    if (r < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    c += r;
    n -= (size_t)r;
  }
  return true;
}

void tune(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  int buf = 8 << 20;
  setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &buf, sizeof buf);
  setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof buf);
}

// writev until every byte of `iov[0..n)` is out (advances over partial writes)
bool writev_all(int fd, iovec *iov, int n) {
  while (n > 0) {
    msghdr m{};
    m.msg_iov = iov;
    m.msg_iovlen = (size_t)(n < IOV_MAX ? n : IOV_MAX);
    ssize_t w = ::sendmsg(fd, &m, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    while (n > 0 && (size_t)w >= iov->iov_len) {
      w -= (ssize_t)iov->iov_len;
      ++iov;
      --n;
    }
    if (n > 0) {
      iov->iov_base = static_cast<char *>(iov->iov_base) + w;
      iov->iov_len -= (size_t)w;
    }
  }
  return true;
}

// ZMTP/3.0 (rfc.zeromq.org 23/ZMTP) constants
constexpr uint8_t kFlagMore = 0x01, kFlagLong = 0x02, kFlagCommand = 0x04;
constexpr size_t kGreetingBytes = 64;
constexpr size_t kMaxCommandBytes = 1 << 20;  // a READY with a few short properties

// frame header: flags + 1-byte or 8-byte big-endian size; returns its length
size_t frame_header(uint8_t *h, uint8_t flags, uint64_t size) {
  if (size > 255) {
    h[0] = flags | kFlagLong;
    const uint64_t be = htobe64(size);
    std::memcpy(h + 1, &be, 8);
    return 9;
  }
  h[0] = flags;
  h[1] = (uint8_t)size;
  return 2;
}

// the rest of a frame header after its flags byte
bool read_size(int fd, uint8_t flags, uint64_t *size) {
  if (flags & kFlagLong) {
    uint64_t be;
    if (!read_all(fd, &be, 8)) return false;
    *size = be64toh(be);
    return true;
  }
  uint8_t s;
  if (!read_all(fd, &s, 1)) return false;
  *size = s;
  return true;
}

bool iequal(const std::string &a, const std::string &b) {
  if (a.size() != b.size()) return false;
  for (size_t i = 0; i < a.size(); ++i)
    if (std::tolower((unsigned char)a[i]) != std::tolower((unsigned char)b[i])) return false;
  return true;
}

void put_prop(std::string &body, const std::string &name, const std::string &value) {
  body.push_back((char)name.size());
  body += name;
  const uint32_t be = htobe32((uint32_t)value.size());
  body.append(reinterpret_cast<const char *>(&be), 4);
  body += value;
}

// the body of a command: name (short string) + data
bool split_command(const std::vector<char> &body, std::string *name, size_t *data_at) {
  if (body.empty()) return false;
  const size_t n = (uint8_t)body[0];
  if (1 + n > body.size()) return false;
  name->assign(body.data() + 1, n);
  *data_at = 1 + n;
  return true;
}

bool read_command(int fd, std::vector<char> *body) {
  uint8_t flags;
  if (!read_all(fd, &flags, 1)) return false;
  uint64_t size;
  if (!(flags & kFlagCommand) || (flags & ~(kFlagLong | kFlagCommand)) || !read_size(fd, flags, &size) ||
      size > kMaxCommandBytes)
    return false;
  body->resize(size);
  return size == 0 || read_all(fd, body->data(), size);
}

}  // namespace

const std::string *PeerInfo::prop(const std::string &name) const {
  for (const auto &p : props)
    if (iequal(p.first, name)) return &p.second;
  return nullptr;
}

bool zmtp_handshake(int fd, const std::string &identity,
                    const std::vector<std::pair<std::string, std::string>> &extra, PeerInfo *peer,
                    std::string *err, double timeout_s) {
  // a peer that connects and then says nothing fails the handshake after
  // timeout_s instead of blocking this thread for ever (libzmq's
  // ZMQ_HANDSHAKE_IVL plays this part); the socket is blocking again after
  struct RecvTimeout {
    int fd;
    RecvTimeout(int f, double s) : fd(f) {
      timeval tv{(time_t)s, (suseconds_t)((s - (double)(time_t)s) * 1e6)};
      setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    }
    ~RecvTimeout() {
      timeval tv{0, 0};
      setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    }
  } guard(fd, timeout_s);
  auto fail = [&](const std::string &why) {
    if (err) *err = "ZMTP handshake: " + why;
    return false;
  };
  auto read_failed = [&](const std::string &what) {
    return fail(errno == EAGAIN || errno == EWOULDBLOCK
                    ? "no " + what + " from the peer within " + std::to_string((int)timeout_s) + " s"
                    : "peer closed during the " + what);
  };
  // greeting: signature, version 3.0, mechanism NULL, as-server 0, filler
  uint8_t g[kGreetingBytes] = {};
  g[0] = 0xFF;
  g[9] = 0x7F;
  g[10] = 3;
  g[11] = 0;
  std::memcpy(g + 12, "NULL", 4);
  if (!write_all(fd, g, sizeof g)) return fail("greeting not sent");
  uint8_t pg[kGreetingBytes];
  errno = 0;
  if (!read_all(fd, pg, sizeof pg)) return read_failed("greeting");
  if (pg[0] != 0xFF || !(pg[9] & 0x01)) return fail("peer is not a ZMTP 2+ endpoint");
  if (pg[10] < 3) return fail("peer speaks ZMTP " + std::to_string(pg[10]) + ".x, need 3.x");
  static const uint8_t null_mech[20] = {'N', 'U', 'L', 'L'};
  if (std::memcmp(pg + 12, null_mech, 20) != 0)
    return fail("peer asks for security mechanism '" +
                std::string(reinterpret_cast<const char *>(pg + 12), strnlen(reinterpret_cast<const char *>(pg + 12), 20)) +
                "', only NULL is spoken");
  // READY, ours then theirs
  std::string body("\x05READY", 6);
  put_prop(body, "Socket-Type", "ROUTER");
  put_prop(body, "Identity", identity);
  for (const auto &p : extra) put_prop(body, p.first, p.second);
  uint8_t h[9];
  iovec iov[2] = {{h, frame_header(h, kFlagCommand, body.size())}, {&body[0], body.size()}};
  if (!writev_all(fd, iov, 2)) return fail("READY not sent");
  std::vector<char> rb;
  errno = 0;
  if (!read_command(fd, &rb)) return errno ? read_failed("READY command") : fail("malformed READY command");
  std::string name;
  size_t at = 0;
  if (!split_command(rb, &name, &at)) return fail("malformed command");
  if (name == "ERROR") {
    const size_t n = at < rb.size() ? (uint8_t)rb[at] : 0;
    return fail("peer sent ERROR: " + std::string(rb.data() + at + 1, std::min(n, rb.size() - at - 1)));
  }
  if (name != "READY") return fail("expected READY, got '" + name + "'");
  PeerInfo info;
  while (at < rb.size()) {
    const size_t nl = (uint8_t)rb[at];
    if (at + 1 + nl + 4 > rb.size()) return fail("truncated READY property");
    std::string pn(rb.data() + at + 1, nl);
    uint32_t vl;
    std::memcpy(&vl, rb.data() + at + 1 + nl, 4);
    vl = be32toh(vl);
    at += 1 + nl + 4;
    if (vl > rb.size() - at) return fail("truncated READY property value");
    info.props.emplace_back(std::move(pn), std::string(rb.data() + at, vl));
    at += vl;
  }
  if (const std::string *t = info.prop("Socket-Type")) info.socket_type = *t;
  if (const std::string *i = info.prop("Identity")) info.identity = *i;
  if (info.socket_type != "ROUTER" && info.socket_type != "DEALER" && info.socket_type != "REQ")
    return fail("a ROUTER cannot talk to a '" + info.socket_type + "' socket");
  if (peer) *peer = std::move(info);
  return true;
}

bool send_frame(int fd, const std::vector<Part> &parts) {
  if (parts.empty() || parts.size() > kMaxParts) return false;
  uint8_t heads[kMaxParts][9];
  iovec iov[2 * kMaxParts];
  int n = 0;
  for (size_t i = 0; i < parts.size(); ++i) {
    const uint8_t flags = i + 1 < parts.size() ? kFlagMore : 0;
    iov[n++] = {heads[i], frame_header(heads[i], flags, parts[i].size)};
    if (parts[i].size) iov[n++] = {const_cast<void *>(parts[i].data), parts[i].size};
  }
  return writev_all(fd, iov, n);
}

bool send_frame_chunked(int fd, const std::vector<Part> &parts, size_t chunk,
                        const std::function<void(size_t)> &ready) {
  if (parts.empty() || parts.size() > kMaxParts || chunk == 0) return false;
  uint8_t heads[kMaxParts][9];
  iovec iov[2 * kMaxParts];
  int n = 0;
  for (size_t i = 0; i < parts.size(); ++i) {
    const bool last = i + 1 == parts.size();
    iov[n++] = {heads[i], frame_header(heads[i], last ? 0 : kFlagMore, parts[i].size)};
    if (!last && parts[i].size) iov[n++] = {const_cast<void *>(parts[i].data), parts[i].size};
  }
  if (!writev_all(fd, iov, n)) return false;  // every header, the parts before the last, its header
  const char *data = static_cast<const char *>(parts.back().data);
  const size_t size = parts.back().size;
  for (size_t k = 0, off = 0; off < size; ++k, off += chunk) {
    ready(k);
    if (!write_all(fd, data + off, size - off < chunk ? size - off : chunk)) return false;
  }
  return true;
}

namespace {
bool recv_frame_impl(int fd, std::vector<RecvPart> &parts, std::vector<std::vector<char>> &scratch,
                     void *(*alloc)(void *ctx, size_t index, size_t size), void *ctx, size_t chunk,
                     const std::function<void(size_t, size_t, size_t)> *landed) {
  parts.clear();
  scratch.resize(kMaxParts);
  for (;;) {
    uint8_t flags;
    if (!read_all(fd, &flags, 1)) return false;
    if (flags & ~(kFlagMore | kFlagLong | kFlagCommand)) return false;  // reserved bits set
    uint64_t size;
    if (!read_size(fd, flags, &size)) return false;
    if (flags & kFlagCommand) {
      // PING / PONG / SUBSCRIBE ...: nothing a ROUTER data path acts on
      if (size > kMaxCommandBytes) return false;
      std::vector<char> body(size);
      if (size && !read_all(fd, body.data(), size)) return false;
      std::string name;
      size_t at = 0;
      if (!split_command(body, &name, &at) || name == "ERROR") return false;
      continue;
    }
    const size_t i = parts.size();
    if (i == kMaxParts) return false;
    void *dst = alloc ? alloc(ctx, i, size) : nullptr;
    if (!dst) {
      scratch[i].resize(size);
      dst = scratch[i].data();
    }
    if (landed) {
      for (size_t off = 0; off < size; off += chunk) {
        const size_t len = size - off < chunk ? size - off : chunk;
        if (!read_all(fd, static_cast<char *>(dst) + off, len)) return false;
        (*landed)(i, off, len);
      }
    } else if (size && !read_all(fd, dst, size)) {
      return false;
    }
    parts.push_back(RecvPart{dst, size});
    if (!(flags & kFlagMore)) return true;
  }
}
}  // namespace

bool recv_frame(int fd, std::vector<RecvPart> &parts, std::vector<std::vector<char>> &scratch,
                void *(*alloc)(void *ctx, size_t index, size_t size), void *ctx) {
  return recv_frame_impl(fd, parts, scratch, alloc, ctx, 0, nullptr);
}

bool recv_frame_chunked(int fd, std::vector<RecvPart> &parts, std::vector<std::vector<char>> &scratch,
                        void *(*alloc)(void *ctx, size_t index, size_t size), void *ctx, size_t chunk,
                        const std::function<void(size_t, size_t, size_t)> &landed) {
  if (chunk == 0) return false;
  return recv_frame_impl(fd, parts, scratch, alloc, ctx, chunk, &landed);
}

int listen_tcp(uint16_t port, std::string *err) {
  const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  if (fd < 0) {
    if (err) *err = std::strerror(errno);
    return -1;
  }
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_ANY);
  a.sin_port = htons(port);
  if (::bind(fd, reinterpret_cast<sockaddr *>(&a), sizeof a) < 0 || ::listen(fd, 64) < 0) {
    if (err) *err = std::string("bind/listen port ") + std::to_string(port) + ": " + std::strerror(errno);
    ::close(fd);
    return -1;
  }
  return fd;
}

int accept_tcp(int listen_fd) {
  for (;;) {
    const int fd = ::accept(listen_fd, nullptr, nullptr);
    if (fd >= 0) {
      tune(fd);
      return fd;
    }
    if (errno != EINTR) return -1;
  }
}

int connect_tcp(const std::string &host_in, uint16_t port, double timeout_s, std::string *err) {
  const std::string host = (host_in == "localhost" || host_in == "local") ? "127.0.0.1" : host_in;
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
  std::string last;
  while (std::chrono::steady_clock::now() < deadline) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    const int g = ::getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res);
    if (g == 0 && res) {
      const int fd = ::socket(res->ai_family, res->ai_socktype, res->ai_protocol);
      if (fd >= 0 && ::connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
        ::freeaddrinfo(res);
        tune(fd);
        return fd;
      }
      last = std::strerror(errno);
      if (fd >= 0) ::close(fd);
      ::freeaddrinfo(res);
    } else {
      last = gai_strerror(g);
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
  if (err) *err = "connect " + host + ":" + std::to_string(port) + ": " + last;
  return -1;
}

void close_fd(int fd) {
  if (fd >= 0) ::close(fd);
}

void shutdown_fd(int fd) {
  if (fd >= 0) ::shutdown(fd, SHUT_RDWR);
}

}  // namespace geeps
