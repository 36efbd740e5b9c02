// TCP framing for libgeeps — see net.hpp.
#include "net.hpp"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

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

}  // namespace

bool send_frame(int fd, const std::vector<Part> &parts) {
  std::vector<char> head(8 + 8 * parts.size());
  const uint32_t magic = kFrameMagic, np = (uint32_t)parts.size();
  std::memcpy(head.data(), &magic, 4);
  std::memcpy(head.data() + 4, &np, 4);
  for (size_t i = 0; i < parts.size(); ++i) {
    const uint64_t len = parts[i].size;
    std::memcpy(head.data() + 8 + 8 * i, &len, 8);
  }
  if (!write_all(fd, head.data(), head.size())) return false;
  for (const Part &p : parts)
    if (p.size && !write_all(fd, p.data, p.size)) return false;
  return true;
}

bool recv_frame(int fd, std::vector<RecvPart> &parts, std::vector<std::vector<char>> &scratch,
                void *(*alloc)(void *ctx, size_t index, size_t size), void *ctx) {
  uint32_t hdr[2];
  if (!read_all(fd, hdr, sizeof hdr)) return false;
  if (hdr[0] != kFrameMagic || hdr[1] > 64) return false;
  std::vector<uint64_t> lens(hdr[1]);
  if (hdr[1] && !read_all(fd, lens.data(), 8 * lens.size())) return false;
  parts.assign(lens.size(), RecvPart{nullptr, 0});
  scratch.resize(lens.size());
  for (size_t i = 0; i < lens.size(); ++i) {
    void *dst = alloc ? alloc(ctx, i, lens[i]) : nullptr;
    if (!dst) {
      scratch[i].resize(lens[i]);
      dst = scratch[i].data();
    }
    if (lens[i] && !read_all(fd, dst, lens[i])) return false;
    parts[i] = RecvPart{dst, lens[i]};
  }
  return true;
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
