#include "hostshare.hpp"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>
#include <random>

#include "gp_reduce.h"

namespace geeps {

namespace {
size_t page_bytes() {
  const long p = sysconf(_SC_PAGESIZE);
  return p > 0 ? (size_t)p : 4096;
}
std::string sys_error(const char *what) { return std::string(what) + ": " + std::strerror(errno); }
constexpr const char *kMemfdName = "geeps-host-oplog";
}  // namespace

std::unique_ptr<SharedHostMem> SharedHostMem::create(size_t bytes, std::string *why) {
  const size_t page = page_bytes();
  const size_t data = (bytes + page - 1) / page * page;
  std::unique_ptr<SharedHostMem> m(new SharedHostMem());
  m->fd_ = memfd_create(kMemfdName, MFD_CLOEXEC);
  if (m->fd_ < 0) {
    *why = sys_error("memfd_create");
    return nullptr;
  }
  if (ftruncate(m->fd_, (off_t)(data + page)) != 0) {
    *why = sys_error("ftruncate");
    return nullptr;
  }
  void *p = mmap(nullptr, data + page, PROT_READ | PROT_WRITE, MAP_SHARED, m->fd_, 0);
  if (p == MAP_FAILED) {
    *why = sys_error("mmap");
    return nullptr;
  }
  m->base_ = p;
  m->bytes_ = data;
  m->map_bytes_ = data + page;
  std::random_device rd;
  for (int i = 0; i < 16; i += 4) {
    const uint32_t r = rd();
    std::memcpy(m->h_.tag + i, &r, 4);
  }
  std::memcpy(static_cast<char *>(p) + data, m->h_.tag, sizeof m->h_.tag);
  m->h_.pid = (int32_t)getpid();
  m->h_.fd = m->fd_;
  m->h_.map_bytes = m->map_bytes_;
  // (unpinned, the buffer still works: its copies go at the pageable rate)
  m->registered_ = gp_host_register(p, data) == GP_OK;
  return m;
}

std::unique_ptr<SharedHostMem> SharedHostMem::open(const HostShareHandle &h, std::string *why) {
  const size_t page = page_bytes();
  if (h.pid <= 0 || h.fd < 0 || h.map_bytes <= page || h.map_bytes % page) {
    *why = "malformed handle";
    return nullptr;
  }
  const std::string path = "/proc/" + std::to_string(h.pid) + "/fd/" + std::to_string(h.fd);
  // only ever a libgeeps host oplog: the descriptor must name one of its memfds
  char target[256] = {};
  const ssize_t len = readlink(path.c_str(), target, sizeof target - 1);
  if (len < 0) {
    *why = sys_error(("open " + path).c_str());
    return nullptr;
  }
  if (std::string(target, (size_t)len).rfind(std::string("/memfd:") + kMemfdName, 0) != 0) {
    *why = path + " is not a libgeeps host oplog (" + std::string(target, (size_t)len) + ")";
    return nullptr;
  }
  const int fd = ::open(path.c_str(), O_RDWR | O_CLOEXEC);
  if (fd < 0) {
    *why = sys_error(("open " + path).c_str());
    return nullptr;
  }
  struct stat st {};
  if (fstat(fd, &st) != 0 || (uint64_t)st.st_size != h.map_bytes) {
    *why = path + " is not the buffer the handle names (size " + std::to_string((long long)st.st_size) +
           ", expected " + std::to_string((unsigned long long)h.map_bytes) + ")";
    ::close(fd);
    return nullptr;
  }
  void *p = mmap(nullptr, h.map_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  ::close(fd);  // (the mapping keeps the memory)
  if (p == MAP_FAILED) {
    *why = sys_error("mmap");
    return nullptr;
  }
  std::unique_ptr<SharedHostMem> m(new SharedHostMem());
  m->base_ = p;
  m->bytes_ = h.map_bytes - page;
  m->map_bytes_ = h.map_bytes;
  if (std::memcmp(static_cast<const char *>(p) + m->bytes_, h.tag, sizeof h.tag) != 0) {
    *why = path + " does not hold the handle's tag";
    return nullptr;
  }
  m->h_ = h;
  m->registered_ = gp_host_register(p, m->bytes_) == GP_OK;
  return m;
}

SharedHostMem::~SharedHostMem() {
  if (registered_) gp_host_unregister(base_);
  if (base_) munmap(base_, map_bytes_);
  if (fd_ >= 0) ::close(fd_);
}

}  // namespace geeps
