// zmtp_peer — one end of libgeeps' wire path (geeps_amd/csrc/geeps/net.cpp)
// as a standalone program, so tests/test_zmtp.py can put a stock libzmq ROUTER
// socket on the other end (a test program: no GPU, no HIP).
//
//   zmtp_peer client <port> <client_id> <server_id> <rows>
//     connects as ROUTER "client-<client_id>" (with libgeeps' X-Geeps-*
//     READY properties), checks the peer is "tablet-<server_id>", pushes one
//     CLOCK_WITH_UPDATES_BATCH [header][RowKey x rows][RowOpVal x rows]
//     (encoder-decoder.cpp:105-124) and checks the READ_ROW_BATCH reply
//     [header][RowKey x rows][RowData x rows] carries 2x the pushed rows.
//   zmtp_peer server <port> <server_id>
//     listens as ROUTER "tablet-<server_id>", accepts one peer, prints its
//     READY properties, answers every CLOCK_WITH_UPDATES_BATCH with that
//     READ_ROW_BATCH (server-encoder-decoder.cpp:228-250) until the peer
//     sends SHUTDOWN or closes.
//
// Row values: update row i, element j = i * 128 + j + 0.25 (exact in fp32).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "net.hpp"
#include "wire.hpp"

using namespace geeps;

namespace {

int fail(const std::string &why) {
  std::fprintf(stderr, "zmtp_peer: %s\n", why.c_str());
  return 1;
}

// ZMTP_PEER_HANDSHAKE_S: the handshake's time limit (default 60 s)
double handshake_s() {
  const char *e = std::getenv("ZMTP_PEER_HANDSHAKE_S");
  return e ? std::atof(e) : 60.0;
}

float update_value(size_t i, size_t j) { return (float)(i * ROW_DATA_SIZE + j) + 0.25f; }

int run_client(uint16_t port, uint32_t client_id, uint32_t server_id, size_t rows) {
  std::string err;
  const int fd = connect_tcp("127.0.0.1", port, 30.0, &err);
  if (fd < 0) return fail(err);
  PeerInfo peer;
  if (!zmtp_handshake(fd, "client-" + std::to_string(client_id),
                      {{"X-Geeps-Ipc", "0"}, {"X-Geeps-Pci-Bus-Id", "0000:00:00.0"}}, &peer, &err,
                      handshake_s()))
    return fail(err);
  std::printf("peer socket_type=%s identity=%s\n", peer.socket_type.c_str(), peer.identity.c_str());
  if (peer.identity != "tablet-" + std::to_string(server_id)) return fail("unexpected server identity");
  cs_clock_with_updates_batch_msg_t h{};
  h.cmd = CLOCK_WITH_UPDATES_BATCH;
  h.client_id = client_id;
  h.clock = 7;
  h.table_id = 0;
  std::vector<RowKey> keys(rows);
  std::vector<RowOpVal> vals(rows);
  for (size_t i = 0; i < rows; ++i) {
    keys[i] = RowKey(0, (row_idx_t)(1000 + i));
    for (size_t j = 0; j < ROW_DATA_SIZE; ++j) vals[i].data[j] = update_value(i, j);
  }
  if (!send_frame(fd, {Part{&h, sizeof h}, Part{keys.data(), rows * sizeof(RowKey)},
                       Part{vals.data(), rows * sizeof(RowOpVal)}}))
    return fail("send failed");
  std::vector<RecvPart> parts;
  std::vector<std::vector<char>> scratch;
  if (!recv_frame(fd, parts, scratch, nullptr, nullptr)) return fail("no reply");
  if (parts.size() != 3 || parts[0].size != sizeof(sc_read_row_batch_msg_t))
    return fail("reply has " + std::to_string(parts.size()) + " parts");
  sc_read_row_batch_msg_t r;
  std::memcpy(&r, parts[0].data, sizeof r);
  if (r.cmd != READ_ROW_BATCH || r.server_id != server_id || r.data_age != 7 || r.table_id != 0)
    return fail("bad reply header");
  if (parts[1].size != rows * sizeof(RowKey) || parts[2].size != rows * sizeof(RowData))
    return fail("bad reply sizes");
  const RowKey *rk = static_cast<const RowKey *>(parts[1].data);
  const RowData *rd = static_cast<const RowData *>(parts[2].data);
  for (size_t i = 0; i < rows; ++i) {
    if (rk[i].table != 0 || rk[i].row != (row_idx_t)(1000 + i)) return fail("bad reply key");
    for (size_t j = 0; j < ROW_DATA_SIZE; ++j)
      if (rd[i].data[j] != 2.0f * update_value(i, j)) return fail("bad reply row");
  }
  cs_clock_msg_t s{};
  s.cmd = SHUTDOWN;
  s.client_id = client_id;
  if (!send_frame(fd, {Part{&s, sizeof s}})) return fail("shutdown send failed");
  close_fd(fd);
  std::printf("client ok rows=%zu\n", rows);
  return 0;
}

int run_server(uint16_t port, uint32_t server_id) {
  std::string err;
  const int lfd = listen_tcp(port, &err);
  if (lfd < 0) return fail(err);
  std::printf("listening\n");
  std::fflush(stdout);
  const int fd = accept_tcp(lfd);
  if (fd < 0) return fail("accept failed");
  PeerInfo peer;
  if (!zmtp_handshake(fd, "tablet-" + std::to_string(server_id), {}, &peer, &err, handshake_s())) return fail(err);
  std::printf("peer socket_type=%s identity=%s\n", peer.socket_type.c_str(), peer.identity.c_str());
  for (const auto &p : peer.props) std::printf("prop %s=%s\n", p.first.c_str(), p.second.c_str());
  std::vector<RecvPart> parts;
  std::vector<std::vector<char>> scratch;
  size_t served = 0;
  while (recv_frame(fd, parts, scratch, nullptr, nullptr)) {
    if (parts.empty() || parts[0].size < sizeof(command_t)) return fail("empty message");
    command_t cmd;
    std::memcpy(&cmd, parts[0].data, sizeof cmd);
    if (cmd == SHUTDOWN) break;
    if (cmd != CLOCK_WITH_UPDATES_BATCH || parts.size() != 3 ||
        parts[0].size != sizeof(cs_clock_with_updates_batch_msg_t))
      return fail("unexpected message");
    cs_clock_with_updates_batch_msg_t h;
    std::memcpy(&h, parts[0].data, sizeof h);
    if (peer.identity != "client-" + std::to_string(h.client_id)) return fail("client id differs from identity");
    const size_t rows = parts[1].size / sizeof(RowKey);
    if (parts[2].size != rows * sizeof(RowOpVal)) return fail("key / row counts differ");
    std::vector<RowData> out(rows);
    const RowOpVal *in = static_cast<const RowOpVal *>(parts[2].data);
    for (size_t i = 0; i < rows; ++i)
      for (size_t j = 0; j < ROW_DATA_SIZE; ++j) out[i].data[j] = in[i].data[j] + in[i].data[j];
    sc_read_row_batch_msg_t r{};
    r.cmd = READ_ROW_BATCH;
    r.server_id = server_id;
    r.data_age = h.clock;
    r.self_clock = h.clock;
    r.table_id = h.table_id;
    if (!send_frame(fd, {Part{&r, sizeof r}, Part{parts[1].data, parts[1].size},
                         Part{out.data(), rows * sizeof(RowData)}}))
      return fail("reply send failed");
    ++served;
  }
  close_fd(fd);
  close_fd(lfd);
  std::printf("server ok served=%zu\n", served);
  return 0;
}

}  // namespace

int main(int argc, char **argv) {
  if (argc >= 6 && !std::strcmp(argv[1], "client"))
    return run_client((uint16_t)std::atoi(argv[2]), (uint32_t)std::atoi(argv[3]), (uint32_t)std::atoi(argv[4]),
                      (size_t)std::atoll(argv[5]));
  if (argc >= 4 && !std::strcmp(argv[1], "server"))
    return run_server((uint16_t)std::atoi(argv[2]), (uint32_t)std::atoi(argv[3]));
  std::fprintf(stderr, "usage: zmtp_peer client <port> <client_id> <server_id> <rows> | server <port> <server_id>\n");
  return 2;
}
