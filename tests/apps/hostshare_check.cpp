// Two-process check of libgeeps' shared host memory (geeps/hostshare.hpp), the
// buffers a same-node server maps to read a client's host-tier rows in place.
//
//   hostshare_check create <floats>
//       creates a buffer, fills float i with i * 0.5, prints one line
//       "<pid> <fd> <map_bytes> <tag hex> <pinned>", then waits for a line on
//       stdin before it exits (the buffer lives until then)
//   hostshare_check open <pid> <fd> <map_bytes> <tag hex> <floats>
//       maps the peer's buffer and checks every float; prints "ok" or the
//       refusal ("refused: ...", exit 3) or the first wrong float (exit 4)
//
// tests/test_hostshare.py drives it (CPU: page-locking needs a GPU and is
// reported, not required).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>

#include "hostshare.hpp"

using geeps::HostShareHandle;
using geeps::SharedHostMem;

static std::string hex(const uint8_t *p, size_t n) {
  std::string s;
  char b[3];
  for (size_t i = 0; i < n; ++i) {
    std::snprintf(b, sizeof b, "%02x", p[i]);
    s += b;
  }
  return s;
}

int main(int argc, char **argv) {
  if (argc >= 3 && std::string(argv[1]) == "create") {
    const size_t n = std::strtoull(argv[2], nullptr, 10);
    std::string why;
    auto m = SharedHostMem::create(n * sizeof(float), &why);
    if (!m) {
      std::cout << "refused: " << why << std::endl;
      return 3;
    }
    float *f = static_cast<float *>(m->data());
    for (size_t i = 0; i < n; ++i) f[i] = (float)i * 0.5f;
    const HostShareHandle &h = m->handle();
    std::cout << h.pid << " " << h.fd << " " << h.map_bytes << " " << hex(h.tag, sizeof h.tag) << " "
              << (m->pinned() ? 1 : 0) << std::endl;
    std::string line;
    std::getline(std::cin, line);
    return 0;
  }
  if (argc >= 7 && std::string(argv[1]) == "open") {
    HostShareHandle h;
    h.pid = std::atoi(argv[2]);
    h.fd = std::atoi(argv[3]);
    h.map_bytes = std::strtoull(argv[4], nullptr, 10);
    const std::string tag = argv[5];
    if (tag.size() != 32) return 2;
    for (int i = 0; i < 16; ++i) h.tag[i] = (uint8_t)std::strtoul(tag.substr(2 * i, 2).c_str(), nullptr, 16);
    const size_t n = std::strtoull(argv[6], nullptr, 10);
    std::string why;
    auto m = SharedHostMem::open(h, &why);
    if (!m) {
      std::cout << "refused: " << why << std::endl;
      return 3;
    }
    if (m->bytes() < n * sizeof(float)) {
      std::cout << "short mapping: " << m->bytes() << std::endl;
      return 4;
    }
    const float *f = static_cast<const float *>(m->data());
    for (size_t i = 0; i < n; ++i)
      if (f[i] != (float)i * 0.5f) {
        std::cout << "float " << i << " = " << f[i] << std::endl;
        return 4;
      }
    std::cout << "ok" << std::endl;
    return 0;
  }
  std::cerr << "usage: hostshare_check create <floats> | open <pid> <fd> <map_bytes> <tag hex> <floats>\n";
  return 2;
}
