// The chunked forms of the wire path (geeps_amd/csrc/geeps/net.cpp) against
// the plain ones over a socketpair, no GPU: send_frame_chunked puts the same
// bytes on the wire as send_frame and calls `ready` once per piece, in order,
// before that piece is written; recv_frame_chunked reads what send_frame wrote
// and calls `landed` for pieces that tile each part exactly.  Prints
// "wire_chunks ok" or the first mismatch, exit status 0 / 1.
#include <sys/socket.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "net.hpp"

using namespace geeps;

static int fail(const char *what) {
  std::printf("wire_chunks FAIL: %s\n", what);
  return 1;
}

int main() {
  for (size_t size : {size_t(0), size_t(1), size_t(7), size_t(64), size_t(1000), size_t(1 << 20) + 3}) {
    for (size_t chunk : {size_t(1), size_t(5), size_t(7), size_t(4096), size_t(1 << 22)}) {
      std::vector<char> head(24), keys(48), rows(size);
      for (size_t i = 0; i < head.size(); ++i) head[i] = (char)(i * 3 + 1);
      for (size_t i = 0; i < keys.size(); ++i) keys[i] = (char)(i * 5 + 2);
      for (size_t i = 0; i < rows.size(); ++i) rows[i] = (char)(i * 7 + size + chunk);
      const std::vector<Part> parts = {{head.data(), head.size()}, {keys.data(), keys.size()}, {rows.data(), rows.size()}};

      // 1. chunked send -> plain receive
      int sv[2];
      if (socketpair(AF_UNIX, SOCK_STREAM, 0, sv)) return fail("socketpair");
      std::vector<size_t> ready_calls;
      bool sent = false;
      std::thread tx([&] {
        sent = send_frame_chunked(sv[0], parts, chunk, [&](size_t k) { ready_calls.push_back(k); });
      });
      std::vector<RecvPart> got;
      std::vector<std::vector<char>> scratch;
      const bool ok = recv_frame(sv[1], got, scratch, nullptr, nullptr);
      tx.join();
      close(sv[0]);
      close(sv[1]);
      if (!sent || !ok) return fail("chunked send / plain receive");
      if (got.size() != 3) return fail("part count");
      for (size_t i = 0; i < 3; ++i)
        if (got[i].size != parts[i].size || (got[i].size && std::memcmp(got[i].data, parts[i].data, got[i].size)))
          return fail("bytes after a chunked send");
      const size_t pieces = (size + chunk - 1) / chunk;
      if (ready_calls.size() != pieces) return fail("ready() calls");
      for (size_t k = 0; k < pieces; ++k)
        if (ready_calls[k] != k) return fail("ready() order");

      // 2. plain send -> chunked receive
      if (socketpair(AF_UNIX, SOCK_STREAM, 0, sv)) return fail("socketpair");
      std::thread tx2([&] { sent = send_frame(sv[0], parts); });
      std::vector<std::vector<size_t>> covered(3);  // next expected offset per part
      std::vector<size_t> next(3, 0);
      bool tiled = true;
      const bool ok2 = recv_frame_chunked(sv[1], got, scratch, nullptr, nullptr, chunk,
                                          [&](size_t i, size_t off, size_t len) {
                                            if (i >= 3 || off != next[i] || len == 0 || len > chunk) tiled = false;
                                            else next[i] += len;
                                          });
      tx2.join();
      close(sv[0]);
      close(sv[1]);
      if (!sent || !ok2) return fail("plain send / chunked receive");
      if (!tiled) return fail("landed() pieces do not tile the parts");
      for (size_t i = 0; i < 3; ++i) {
        if (next[i] != parts[i].size) return fail("landed() coverage");
        if (got[i].size != parts[i].size || (got[i].size && std::memcmp(got[i].data, parts[i].data, got[i].size)))
          return fail("bytes after a chunked receive");
      }
    }
  }
  std::printf("wire_chunks ok\n");
  return 0;
}
