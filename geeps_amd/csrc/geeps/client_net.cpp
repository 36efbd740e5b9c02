// ClientLib's network side: the ZMTP connections, the server side of each
// client connection and the client side of each server connection (frames,
// IPC references, NACK / resend), the refresh replies.  Reference:
// src/client/encoder-decoder.cpp, src/server/server-encoder-decoder.cpp,
// src/client/clientlib-cbk.cpp.
#include "client.hpp"

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <fstream>
#include <iostream>
#include <set>
#include <sstream>
#include <unordered_set>

#include "check.hpp"
#include "net.hpp"
#include "client_internal.hpp"

namespace geeps {

using namespace client_detail;

uint16_t ClientLib::port_of(uint32_t process, uint32_t channel) const {
  // The reference binds tcp_base_port + channel on every host and ignores
  // port_list (clientlib.cpp:57-60, 111-112; server-entry.cpp:56-57); honouring
  // port_list lets several processes share one host (BASELINE config 1).
  const uint32_t base = config_.port_list.empty() ? config_.tcp_base_port : config_.port_list[process];
  return (uint16_t)(base + channel);
}

void ClientLib::start_network() {
  if (num_processes_ == 1) return;
  // 1. listen: this process's tablet server of every channel
  for (auto &chp : channels_) {
    std::string err;
    chp->listen_fd = listen_tcp(port_of(process_id_, chp->id), &err);
    GP_CHECK_MSG(chp->listen_fd >= 0, err);
  }
  accept_thread_ = std::thread([this] {
    GP_CALL(gp_set_device(device_));
    for (auto &chp : channels_) server_accept_loop(*chp, (int)num_processes_ - 1);
  });
  // 2. connect: this process's client to every remote server
  for (auto &chp : channels_) {
    Channel &ch = *chp;
    for (uint32_t s = 0; s < num_processes_; ++s) {
      if (s == process_id_) continue;
      std::string err;
      const int fd = connect_tcp(config_.host_list[s], port_of(s, ch.id), connect_timeout_s(), &err);
      GP_CHECK_MSG(fd >= 0, err);
      // ZMTP READY as the reference's client ROUTER ("client-<i>",
      // clientlib.cpp:107); the server must answer as "tablet-<s>"
      PeerInfo peer;
      // (the server's accept thread may still be taking an earlier channel's
      // connections from slower processes: as long as a connect may take)
      GP_CHECK_MSG(zmtp_handshake(fd, "client-" + std::to_string(process_id_), hello_props(s), &peer, &err,
                                  connect_timeout_s()),
                   err << " (server " << s << ", channel " << ch.id << ")");
      GP_CHECK_MSG(peer.identity == "tablet-" + std::to_string(s),
                   "port " << port_of(s, ch.id) << " answered as '" << peer.identity << "', expected tablet-" << s);
      ch.server_fd[s] = fd;
      ch.client_readers.emplace_back([this, &ch, s, fd] { client_reader(ch, s, fd); });
    }
  }
  accept_thread_.join();
}

void ClientLib::server_accept_loop(Channel &ch, int expected) {
  for (int i = 0; i < expected; ++i) {
    const int fd = accept_tcp(ch.listen_fd);
    GP_CHECK_MSG(fd >= 0, "accept failed on channel " << ch.id);
    // ZMTP READY as the reference's server ROUTER ("tablet-<i>",
    // server-entry.cpp:66); the peer names itself "client-<i>"
    PeerInfo peer;
    std::string err;
    GP_CHECK_MSG(zmtp_handshake(fd, "tablet-" + std::to_string(process_id_), {}, &peer, &err,
                                connect_timeout_s()),
                 err << " (channel " << ch.id << ")");
    uint32_t cid = ~0u;
    {
      const std::string &id = peer.identity;
      char *end = nullptr;
      if (id.compare(0, 7, "client-") == 0 && id.size() > 7) cid = (uint32_t)std::strtoul(id.c_str() + 7, &end, 10);
      GP_CHECK_MSG(end && *end == 0, "connection from '" << id << "', expected a client-<i> identity");
    }
    GP_CHECK_LT(cid, num_processes_);
    GP_CHECK_MSG(ch.client_fd[cid] < 0, "duplicate client " << cid);
    ch.client_fd[cid] = fd;
    const std::string *ipc = peer.prop("X-Geeps-Ipc"), *bus = peer.prop("X-Geeps-Pci-Bus-Id");
    ch.ipc_client[cid] = ipc && *ipc == "1" && ipc_to(cid);
    // process cid hosts client cid and server cid on the same GPU, so one
    // READY decides both directions
    ch.other_gpu[cid] = !bus || *bus != pci_bus_id_;
    auto staged = [&](int mode) { return ipc_to(cid) && (mode == 1 || (mode < 0 && ch.other_gpu[cid])); };
    ch.stage_from[cid] = staged(stage_updates_mode_);
    ch.stage_refresh_from[cid] = staged(stage_refresh_mode_);
    ch.server_readers.emplace_back([this, &ch, cid, fd] { server_reader(ch, cid, fd); });
  }
}

namespace {
// A frame a reader holds back while it awaits a resend (IPC recovery,
// wire.hpp): its parts copied, part 2's rows in a pinned buffer of its own.
struct HeldFrame {
  std::vector<std::vector<char>> parts;
  std::shared_ptr<PinnedArray<float>> rows;  // part 2, when it had bytes
  size_t rows_bytes = 0;
  std::vector<RecvPart> view() {
    std::vector<RecvPart> v;
    for (size_t i = 0; i < parts.size(); ++i)
      v.push_back(i == 2 && rows ? RecvPart{rows->data(), rows_bytes} : RecvPart{parts[i].data(), parts[i].size()});
    return v;
  }
};

// Receives one whole frame into a HeldFrame of its own (part 2 into fresh
// pinned memory).  False at EOF.
bool recv_held(int fd, HeldFrame *f) {
  std::vector<RecvPart> parts;
  std::vector<std::vector<char>> scratch;
  auto alloc = [](void *c, size_t i, size_t size) -> void * {
    auto *h = static_cast<HeldFrame *>(c);
    if (i != 2 || size == 0) return nullptr;
    h->rows = std::make_shared<PinnedArray<float>>((size + 3) / 4);
    h->rows_bytes = size;
    return h->rows->data();
  };
  if (!recv_frame(fd, parts, scratch, alloc, f)) return false;
  for (size_t i = 0; i < parts.size(); ++i) {
    const char *d = static_cast<const char *>(parts[i].data);
    f->parts.emplace_back(i == 2 && f->rows ? std::vector<char>() : std::vector<char>(d, d + parts[i].size));
  }
  return true;
}
}  // namespace

// Server side of a client connection: CLOCK_WITH_UPDATES_BATCH / CLOCK frames
// (ClientServerDecode::decode_msg, server-encoder-decoder.cpp:153-183).
void ClientLib::server_reader(Channel &ch, uint32_t client_id, int fd) {
  GP_CALL(gp_set_device(device_));
  PinnedPool pool;
  struct Ctx {
    PinnedPool *pool;
    std::shared_ptr<PinnedArray<float>> rows;
  } ctx{&pool, nullptr};
  auto alloc = [](void *c, size_t i, size_t size) -> void * {
    auto *x = static_cast<Ctx *>(c);
    if (i != 2) return nullptr;
    x->rows = x->pool->get((size + 3) / 4);
    return x->rows->data();
  };
  std::vector<RecvPart> parts;
  std::vector<std::vector<char>> scratch;
  std::deque<HeldFrame> held;  // frames after a NACKed one, until its resend
  PinnedArray<float> resend_buf;
  std::unique_ptr<Stream> resend_stream;
  // false: the connection's last frame
  std::function<bool(const std::vector<RecvPart> &, const std::shared_ptr<PinnedArray<float>> &)> handle =
      [&](const std::vector<RecvPart> &parts, const std::shared_ptr<PinnedArray<float>> &host_rows) -> bool {
    GP_CHECK(!parts.empty() && parts[0].size >= 1);
    const command_t cmd = *static_cast<const command_t *>(parts[0].data);
    if (cmd == CLOCK_WITH_UPDATES_BATCH) {
      GP_CHECK(parts.size() >= 3 && parts.size() <= 5 && parts[0].size == sizeof(cs_clock_with_updates_batch_msg_t));
      cs_clock_with_updates_batch_msg_t h;
      std::memcpy(&h, parts[0].data, sizeof h);
      GP_CHECK_EQ(h.client_id, client_id);
      size_t n = parts[1].size / sizeof(RowKey);
      UpdateBatch b;
      b.client_id = h.client_id;
      b.clock = h.clock;
      b.table_id = h.table_id;
      auto take_keys = [&](const RecvPart &k) {
        auto keys = std::make_shared<std::vector<RowKey>>(k.size / sizeof(RowKey));
        std::memcpy(keys->data(), k.data, k.size);
        b.keys = keys->data();
        b.keys_owner = keys;
      };
      if (n) take_keys(parts[1]);
      std::shared_ptr<PinnedArray<float>> rows = host_rows;
      if (parts.size() >= 4) {
        // Same-node client: the rows stay in its oplog, mapped here over IPC;
        // a table with a host tier sends its host-tier rows first, in the
        // frame, or (a 5th part) names them in its shared host oplog
        GP_CHECK(parts[3].size == sizeof(IpcRowsRef) && parts[2].size % kRowBytes == 0);
        IpcRowsRef ref;
        std::memcpy(&ref, parts[3].data, sizeof ref);
        GP_CHECK(ref.bytes % kRowBytes == 0);
        HostRowsRef href{};
        const bool host_ref = parts.size() == 5;
        if (host_ref) {
          GP_CHECK(parts[4].size == sizeof(HostRowsRef) && parts[2].size == 0);
          std::memcpy(&href, parts[4].data, sizeof href);
          GP_CHECK(href.bytes % kRowBytes == 0 && href.bytes > 0);
        }
        const size_t head_bytes = host_ref ? href.bytes : parts[2].size;
        const size_t head = head_bytes / kRowBytes;
        if (n) GP_CHECK_EQ(head_bytes + ref.bytes, n * kRowBytes);
        n = head + ref.bytes / kRowBytes;  // key part omitted after the first message
        if (head && !host_ref) {
          b.split = head;
          b.host_head = rows->data();
          b.head_keepalive = rows;
        }
        uint32_t unmapped = 0;  // kNackDevice | kNackHost
        if (host_ref) {
          auto &hmapped = ch.host_oplogs[client_id];
          if (href.has_handle) {
            hmapped.erase(href.buffer_id);
            std::string why;
            std::shared_ptr<SharedHostMem> m = SharedHostMem::open(href.handle, &why);
            if (m) {
              hmapped[href.buffer_id] = m;
            } else {
              unmapped |= kNackHost;
              std::cerr << "libgeeps: server " << process_id_ << " ch " << ch.id << " could not map host oplog "
                        << href.buffer_id << " of client " << client_id << " (" << why
                        << "); asking for the rows by socket\n";
            }
          }
          if (!unmapped) {
            auto it = hmapped.find(href.buffer_id);
            GP_CHECK_MSG(it != hmapped.end(), "unmapped host oplog " << href.buffer_id);
            GP_CHECK_LE(href.offset + href.bytes, it->second->bytes());
            b.split = head;
            b.host_head =
                reinterpret_cast<const float *>(static_cast<const char *>(it->second->data()) + href.offset);
            b.head_keepalive = it->second;
          }
        }
        auto &mapped = ch.ipc_oplogs[client_id];
        bool ok = true;
        if (ref.has_handle) {
          auto old = mapped.find(ref.buffer_id);
          if (old != mapped.end()) {
            ch.ipc_parked[client_id].push_back(old->second);  // closed at Shutdown (client.hpp)
            mapped.erase(old);
          }
          void *p = nullptr;
          ok = gp_ipc_open_handle(&p, ref.handle) == GP_OK;
          if (ok) {
            mapped[ref.buffer_id] = p;
            if (ipc_log())
              std::cerr << "libgeeps ipc map oplog: server " << process_id_ << " ch " << ch.id << " client "
                        << client_id << " buffer " << ref.buffer_id << " -> " << p << ": "
                        << ipc_describe(ref.handle) << "\n";
          } else {
            std::cerr << "libgeeps: server " << process_id_ << " ch " << ch.id << " could not map oplog buffer "
                      << ref.buffer_id << " of client " << client_id << " (" << gp_last_error()
                      << "); asking for the rows by socket\n";
          }
        }
        if (!ok) unmapped |= kNackDevice;
        if (!unmapped) {
          if (ref.bytes) {  // (none: the table's rows are all in the host tier)
            auto it = mapped.find(ref.buffer_id);
            GP_CHECK_MSG(it != mapped.end(), "unmapped oplog buffer " << ref.buffer_id);
            b.device_rows = reinterpret_cast<const float *>(static_cast<const char *>(it->second) + ref.offset);
            b.stage = ch.stage_from[client_id];
          }
        } else {
          // NACK, then hold the client's later frames back until the slice
          // comes again as a socket frame (the client sends it as soon as its
          // reader sees the NACK)
          OplogNackMsg m{};
          m.cmd = kCmdOplogNack;
          m.server_id = process_id_;
          m.table_id = h.table_id;
          m.unmapped = unmapped;
          m.clock = h.clock;
          m.buffer_id = ref.buffer_id;
          GP_CHECK_MSG(send_to_client(ch, client_id, {Part{&m, sizeof m}}),
                       "oplog NACK to client " << client_id << " failed");
          {
            std::lock_guard<std::mutex> lk(stats_mu_);
            stats_.nr_ipc_nack_sent++;
          }
          for (;;) {
            HeldFrame f;
            GP_CHECK_MSG(recv_held(fd, &f), "client " << client_id << " closed before resending clock "
                                                        << h.clock << " of table " << h.table_id);
            cs_clock_with_updates_batch_msg_t r{};
            if (f.parts.size() == 3 && f.parts[0].size() == sizeof r) std::memcpy(&r, f.parts[0].data(), sizeof r);
            if (f.parts.size() == 3 && r.cmd == CLOCK_WITH_UPDATES_BATCH && r.clock == h.clock &&
                r.table_id == h.table_id) {
              const std::vector<RecvPart> v = f.view();
              GP_CHECK_EQ(v[1].size / sizeof(RowKey), n);
              GP_CHECK_EQ(v[2].size, n * kRowBytes);
              take_keys(v[1]);  // (the resend always carries the keys)
              rows = f.rows;
              b.split = 0;  // (all its rows, host-tier ones first, in the frame)
              b.host_head = nullptr;
              b.head_keepalive.reset();
              break;
            }
            // the client's own NACK of a version, and its releases, do not
            // wait behind the resend (its reader may be awaiting this server's
            // resend at the same time: holding them back would deadlock)
            const command_t fc = f.parts.empty() || f.parts[0].empty() ? 0 : (command_t)f.parts[0][0];
            if (fc == kCmdVersionNack || fc == kCmdRefreshAck) {
              handle(f.view(), f.rows);
              continue;
            }
            held.push_back(std::move(f));
          }
        }
      } else {
        GP_CHECK_EQ(parts[2].size, n * kRowBytes);
      }
      if (!b.device_rows) b.host_rows = rows;
      b.num_rows = n;
      ch.server->post_updates(std::move(b));
    } else if (cmd == kCmdRefreshAck) {
      GP_CHECK(parts.size() == 1 && parts[0].size == sizeof(RefreshAckMsg));
      RefreshAckMsg a;
      std::memcpy(&a, parts[0].data, sizeof a);
      GP_CHECK_EQ(a.client_id, client_id);
      ch.server->release(client_id, a.table_id, a.version);
    } else if (cmd == kCmdVersionNack) {
      GP_CHECK(parts.size() == 1 && parts[0].size == sizeof(VersionNackMsg));
      VersionNackMsg m;
      std::memcpy(&m, parts[0].data, sizeof m);
      GP_CHECK_EQ(m.client_id, client_id);
      if (!resend_stream) resend_stream = std::make_unique<Stream>();
      resend_version(ch, client_id, m, resend_buf, *resend_stream);
    } else if (cmd == CLOCK) {
      GP_CHECK(parts.size() == 1 && parts[0].size == sizeof(cs_clock_msg_t));
      cs_clock_msg_t h;
      std::memcpy(&h, parts[0].data, sizeof h);
      ch.server->post_clock(h.client_id, h.clock, h.table_id);
    } else if (cmd == SHUTDOWN) {
      // The client sends nothing after this (shutdown handshake) and reads no
      // more: later refreshes to it are dropped and its holds end here.
      {
        std::lock_guard<std::mutex> lk(ch.ipc_mu);
        ch.client_done[client_id] = 1;
      }
      ch.server->release_all(client_id);
      ch.server->post_shutdown(client_id);
      // its last frame, kCmdReaderDone, comes once it has handled this
      // server's SHUTDOWN (shutdown()): this process waits for it
    } else if (cmd == kCmdReaderDone) {
      return false;
    } else {
      GP_CHECK_MSG(false, "server received unknown command " << (int)cmd);
    }
    return true;
  };
  for (;;) {
    if (!held.empty()) {
      HeldFrame f = std::move(held.front());
      held.pop_front();
      if (!handle(f.view(), f.rows)) break;
      continue;
    }
    ctx.rows.reset();
    if (!recv_frame(fd, parts, scratch, alloc, &ctx)) break;
    if (!handle(parts, ctx.rows)) break;
  }
}

// A client NACKed master version m.version (it could not map it): the same
// refresh again as a socket frame from the version's rows (the client still
// holds the version, so nothing wrote it), then the hold goes back and the
// handle counts as not sent.
void ClientLib::resend_version(Channel &ch, uint32_t c, const VersionNackMsg &m, PinnedArray<float> &buf,
                               const Stream &st) {
  const float *rows = nullptr;
  size_t n = 0;
  const RowKey *keys = nullptr;
  ch.server->held_version(c, m.table_id, m.version, &rows, &n, &keys);
  const size_t floats = n * ROW_DATA_SIZE;
  if (buf.size() < floats) buf.resize(floats);
  if (floats) GP_CALL(gp_memcpy_async(buf.data(), rows, floats * sizeof(float), st.get()));
  st.sync();
  sc_read_row_batch_msg_t h{};
  h.cmd = READ_ROW_BATCH;
  h.server_id = process_id_;
  h.data_age = m.data_age;
  h.self_clock = m.self_clock;
  h.table_id = m.table_id;
  GP_CHECK_MSG(send_to_client(ch, c, {Part{&h, sizeof h}, Part{keys, n * sizeof(RowKey)},
                                      Part{buf.data(), floats * sizeof(float)}}),
               "resend to client " << c << " failed");
  {
    std::lock_guard<std::mutex> lk(ch.ipc_mu);
    ch.version_sent[c][m.table_id].erase(m.version);
  }
  ch.server->release(c, m.table_id, m.version);
  std::lock_guard<std::mutex> lk(stats_mu_);
  stats_.nr_ipc_resent++;
}

// A server NACKed this client's oplog slice of (table, clock): the oplog is
// still here (reclaimed only once every server's refresh covers the clock,
// and this server's cannot before it has these rows), so the slice goes again
// as an ordinary socket frame; push_updates exports a fresh buffer in place of
// the NACKed one on its next use, or, when it was the shared host oplog the
// server could not map, sends that server the host-tier rows in the frame.
void ClientLib::resend_oplog(Channel &ch, uint32_t s, const OplogNackMsg &m, PinnedArray<float> &buf,
                             const Stream &st) {
  std::shared_ptr<DeviceArray<float>> oplog;
  std::shared_ptr<HostBuf> hoplog;  // with a host tier: its rows go first
  std::shared_ptr<const std::vector<RowKey>> keys;
  const RowKey *key0 = nullptr;
  size_t a = 0, n = 0, ca = 0, cn = 0;
  {
    std::lock_guard<std::mutex> lk(ch.mu);
    GP_CHECK_LT(m.table_id, ch.tables.size());
    ParamCache &pc = ch.tables[m.table_id];
    auto it = pc.oplog.find(m.clock);
    if (pc.num_rows || it != pc.oplog.end()) {  // (a table wholly in the host tier has no HBM oplog)
      GP_CHECK_MSG(it != pc.oplog.end(), "server " << s << " NACKed clock " << m.clock << " of table "
                                                   << m.table_id << ", whose oplog is gone");
      oplog = it->second;
    }
    a = pc.server_row_start[s];
    n = pc.server_num_rows[s];
    if (pc.cpu.num_rows) {
      auto hit = pc.cpu.oplog.find(m.clock);
      GP_CHECK_MSG(hit != pc.cpu.oplog.end(), "NACKed clock " << m.clock << ": its host oplog is gone");
      hoplog = hit->second;
      ca = pc.cpu.server_row_start[s];
      cn = pc.cpu.server_num_rows[s];
      keys = pc.frame_keys[s];
      key0 = keys->data();
    } else {
      keys = pc.row_keys;
      key0 = keys->data() + a;
    }
    if (m.unmapped != kNackHost) pc.ipc_nacked.emplace_back((size_t)(m.buffer_id & 0xffffffffu), s);
    if (m.unmapped & kNackHost) ch.host_share_off[s] = 1;  // its host-tier rows go in the frame from now on
  }
  if (m.unmapped & kNackHost) {
    std::lock_guard<std::mutex> lk(stats_mu_);
    stats_.nr_host_share_refused++;
  }
  const size_t floats = (cn + n) * ROW_DATA_SIZE;
  if (buf.size() < floats) buf.resize(floats);
  if (cn) std::memcpy(buf.data(), hoplog->data() + ca * ROW_DATA_SIZE, cn * kRowBytes);
  if (n)
    GP_CALL(gp_memcpy_async(buf.data() + cn * ROW_DATA_SIZE, oplog->data() + a * ROW_DATA_SIZE, n * kRowBytes,
                            st.get()));
  st.sync();
  cs_clock_with_updates_batch_msg_t h{};
  h.cmd = CLOCK_WITH_UPDATES_BATCH;
  h.client_id = process_id_;
  h.clock = m.clock;
  h.table_id = m.table_id;
  {
    // (also after this client's SHUTDOWN: the server's reader awaits this
    // frame and holds the SHUTDOWN back behind it)
    std::lock_guard<std::mutex> lk(*ch.server_send_mu[s]);
    GP_CHECK_MSG(send_frame(ch.server_fd[s], {Part{&h, sizeof h}, Part{key0, (cn + n) * sizeof(RowKey)},
                                              Part{buf.data(), floats * sizeof(float)}}),
                 "resend to server " << s << " failed");
  }
  std::lock_guard<std::mutex> lk(stats_mu_);
  stats_.nr_ipc_resent++;
}

bool ClientLib::send_to_client(Channel &ch, uint32_t c, const std::vector<Part> &parts) {
  std::lock_guard<std::mutex> lk(*ch.client_send_mu[c]);
  return send_frame(ch.client_fd[c], parts);
}

bool ClientLib::ipc_export(void *handle, void *base, int kind) {
  const bool fault = ipc_fault_ && !ipc_fault_used_[kind].exchange(true);
  if (fault && ipc_fault_ == 2) {
    std::cerr << "libgeeps: GEEPS_TEST_IPC_FAULT=refuse: export " << (kind ? "of a master version" : "of an oplog")
              << " refused\n";
    return false;
  }
  if (gp_ipc_get_handle(handle, base) != GP_OK) {
    std::cerr << "libgeeps: IPC export of " << base << " refused (" << gp_last_error()
              << "); the rows go by socket\n";
    return false;
  }
  if (fault) {
    // the tag's last byte (gp_reduce.hip IpcHandleOut: the runtime's 64-B
    // handle, the tag's offset, then the 16-B tag): the importer's check fails
    static_cast<uint8_t *>(handle)[64 + 8 + 15] ^= 0x5a;
    std::cerr << "libgeeps: GEEPS_TEST_IPC_FAULT=tag: corrupted the tag of an exported "
              << (kind ? "master version" : "oplog") << "\n";
  }
  return true;
}


// Client side of a server connection: READ_ROW_BATCH replies
// (ServerClientDecode::read_row_batch, client/encoder-decoder.cpp:228-251).
void ClientLib::client_reader(Channel &ch, uint32_t server_id, int fd) {
  GP_CALL(gp_set_device(device_));
  PinnedArray<float> buf;
  std::vector<RecvPart> parts;
  std::vector<std::vector<char>> scratch;
  // A socket refresh's rows go on to HBM piece by piece as they come off the
  // socket (into `landing`, this reader's own buffer: one refresh at a time),
  // so the host-to-device copy overlaps the receive; recv_row_batch then
  // copies device to device under the channel lock.
  DeviceArray<float> landing;
  Stream h2d;
  auto landed = [&](size_t i, size_t off, size_t len) {
    if (i != 2) return;
    GP_CALL(gp_memcpy_async(reinterpret_cast<char *>(landing.data()) + off,
                            reinterpret_cast<const char *>(buf.data()) + off, len, h2d.get()));
  };
  auto alloc_landing = [](void *c, size_t i, size_t size) -> void * {
    auto *ctx = static_cast<std::pair<PinnedArray<float> *, DeviceArray<float> *> *>(c);
    if (i != 2) return nullptr;
    if (ctx->first->size() * 4 < size) ctx->first->resize((size + 3) / 4);
    if (ctx->second->size() * 4 < size) ctx->second->resize((size + 3) / 4);
    return ctx->first->data();
  };
  std::pair<PinnedArray<float> *, DeviceArray<float> *> ctx{&buf, &landing};
  static const bool stream_recv = [] {
    const char *e = std::getenv("GEEPS_STREAM_RECV");
    return !e || std::atoi(e) != 0;
  }();
  auto alloc_pinned = [](void *c, size_t i, size_t size) -> void * {
    auto *b = static_cast<std::pair<PinnedArray<float> *, DeviceArray<float> *> *>(c)->first;
    if (i != 2) return nullptr;
    if (b->size() * 4 < size) b->resize((size + 3) / 4);
    return b->data();
  };
  std::deque<HeldFrame> held;  // frames after a NACKed refresh, until its resend
  PinnedArray<float> resend_buf;
  auto ack_all = [&](uint32_t table, const std::vector<int> &released) {
    for (int v : released) {
      RefreshAckMsg a{};
      a.cmd = kCmdRefreshAck;
      a.client_id = process_id_;
      a.table_id = table;
      a.version = v;
      ack_to_server(ch, server_id, a);
    }
  };
  // false: the server's SHUTDOWN (its last frame).  `in_landing`: part 2's
  // rows were streamed into `landing` (else they are in host memory at
  // parts[2].data).
  std::function<bool(const std::vector<RecvPart> &, bool)> handle = [&](const std::vector<RecvPart> &parts,
                                                                         bool in_landing) {
    GP_CHECK(!parts.empty() && parts[0].size >= 1);
    const command_t cmd = *static_cast<const command_t *>(parts[0].data);
    if (cmd == SHUTDOWN) {
      // The server sends nothing more.  Every frame it sent is handled; once
      // no queued device work reads its memory, say so: it waits for that
      // before its process exits and frees what its handles named.
      GP_CALL(gp_device_synchronize());
      reader_done_to_server(ch, server_id);
      return false;
    }
    if (cmd == kCmdOplogNack) {
      GP_CHECK(parts.size() == 1 && parts[0].size == sizeof(OplogNackMsg));
      OplogNackMsg m;
      std::memcpy(&m, parts[0].data, sizeof m);
      GP_CHECK_EQ(m.server_id, server_id);
      resend_oplog(ch, server_id, m, resend_buf, h2d);
      return true;
    }
    if (reader_delay_us_ > 0) std::this_thread::sleep_for(std::chrono::microseconds(reader_delay_us_));
    GP_CHECK((parts.size() == 3 || parts.size() == 4) &&
             parts[0].size == sizeof(sc_read_row_batch_msg_t));
    sc_read_row_batch_msg_t h;
    std::memcpy(&h, parts[0].data, sizeof h);
    GP_CHECK_EQ(h.cmd, (command_t)READ_ROW_BATCH);
    GP_CHECK_EQ(h.server_id, server_id);
    GP_CHECK_LT(h.table_id, config_.num_tables);
    if (parts.size() == 4) {
      // Same-node server: the shard is one of its master versions, read in
      // place through an IPC mapping of that version's buffer.
      GP_CHECK(parts[3].size == sizeof(IpcRefreshVersion));
      IpcRefreshVersion rv;
      std::memcpy(&rv, parts[3].data, sizeof rv);
      GP_CHECK(rv.version >= 0);
      void *ptr = nullptr;
      bool ok = true;
      {
        std::lock_guard<std::mutex> lk(ch.mu);
        auto &mapped = ch.tables[h.table_id].server_versions[server_id];
        if (rv.has_handle) {
          GP_CHECK_MSG(!mapped.count(rv.version), "version " << rv.version << " mapped twice");
          ok = gp_ipc_open_handle(&ptr, rv.handle) == GP_OK;
          if (ok) mapped[rv.version] = ptr;
          if (ok && ipc_log())
            std::cerr << "libgeeps ipc map version: client " << process_id_ << " ch " << ch.id << " server "
                      << server_id << " table " << h.table_id << " version " << rv.version << " rows "
                      << rv.num_rows << " -> " << ptr << ": " << ipc_describe(rv.handle) << "\n";
        } else {
          auto it = mapped.find(rv.version);
          GP_CHECK_MSG(it != mapped.end(), "unmapped master version " << rv.version);
          ptr = it->second;
        }
      }
      if (!ok) {
        // NACK: the server sends this refresh again as a socket frame; hold
        // later frames back until it arrives, then take it as a copy
        std::cerr << "libgeeps: client " << process_id_ << " ch " << ch.id << " could not map master version "
                  << rv.version << " of server " << server_id << " (" << gp_last_error()
                  << "); asking for the refresh by socket\n";
        VersionNackMsg m{};
        m.cmd = kCmdVersionNack;
        m.client_id = process_id_;
        m.table_id = h.table_id;
        m.version = rv.version;
        m.data_age = h.data_age;
        m.self_clock = h.self_clock;
        {
          std::lock_guard<std::mutex> lk(*ch.server_send_mu[server_id]);
          // after this client's SHUTDOWN it reads nothing more, and the server
          // has let go of its holds: the refresh is dropped
          if (ch.server_shut[server_id]) return true;
          GP_CHECK_MSG(send_frame(ch.server_fd[server_id], {Part{&m, sizeof m}}),
                       "version NACK to server " << server_id << " failed");
        }
        {
          std::lock_guard<std::mutex> lk(stats_mu_);
          stats_.nr_ipc_nack_sent++;
        }
        for (;;) {
          HeldFrame f;
          GP_CHECK_MSG(recv_held(fd, &f), "server " << server_id << " closed before resending table "
                                                    << h.table_id << " at data age " << h.data_age);
          sc_read_row_batch_msg_t r{};
          if (f.parts.size() == 3 && f.parts[0].size() == sizeof r) std::memcpy(&r, f.parts[0].data(), sizeof r);
          if (f.parts.size() == 3 && r.cmd == READ_ROW_BATCH && r.table_id == h.table_id &&
              r.data_age == h.data_age) {
            const std::vector<RecvPart> v = f.view();
            GP_CHECK_EQ(v[2].size, rv.num_rows * kRowBytes);
            ack_all(h.table_id, recv_row_batch(ch.id, h.server_id, h.table_id, h.data_age, h.self_clock,
                                               static_cast<const float *>(v[2].data), rv.num_rows, -1, nullptr,
                                               static_cast<const float *>(v[2].data)));
            break;
          }
          // the server's NACK of an oplog does not wait behind the resend
          // (its reader may be awaiting this client's resend at the same time)
          if (!f.parts.empty() && !f.parts[0].empty() && (command_t)f.parts[0][0] == kCmdOplogNack) {
            handle(f.view(), false);
            continue;
          }
          held.push_back(std::move(f));
        }
        return true;
      }
      const float *src = static_cast<const float *>(ptr);
      if (ch.stage_refresh_from[server_id] && rv.num_rows) {
        // A staged refresh (a server on another GPU): the peer copy over xGMI
        // goes to this reader's landing buffer first, on its own stream and
        // outside the channel lock, so the refreshes of several peers come
        // over their links at once; recv_row_batch then swaps it into the
        // cache under the lock (ParamCache::shard_buf).  (The version stays
        // held until then.)
        const size_t bytes = rv.num_rows * kRowBytes;
        if (landing.size() * sizeof(float) < bytes) landing.resize(bytes / sizeof(float));
        GP_CALL(gp_memcpy_async(landing.data(), src, bytes, h2d.get()));
        h2d.sync();
        src = landing.data();
      }
      ack_all(h.table_id, recv_row_batch(ch.id, h.server_id, h.table_id, h.data_age, h.self_clock, src,
                                         rv.num_rows, rv.version, src == landing.data() ? &landing : nullptr));
      return true;
    }
    const size_t n = parts[1].size / sizeof(RowKey);
    GP_CHECK_EQ(parts[2].size, n * kRowBytes);
    if (in_landing) h2d.sync();  // every piece's copy into `landing` has landed
    // (a socket refresh may replace a shard this client read in place, when the
    // server's export of its version was refused: those versions go back)
    ack_all(h.table_id,
            recv_row_batch(ch.id, h.server_id, h.table_id, h.data_age, h.self_clock,
                           n && in_landing ? landing.data() : static_cast<const float *>(parts[2].data), n, -1,
                           n && in_landing ? &landing : nullptr, static_cast<const float *>(parts[2].data)));
    return true;
  };
  for (;;) {
    if (!held.empty()) {
      HeldFrame f = std::move(held.front());
      held.pop_front();
      if (!handle(f.view(), false)) break;
      continue;
    }
    if (stream_recv ? !recv_frame_chunked(fd, parts, scratch, alloc_landing, &ctx, kWireChunk, landed)
                    : !recv_frame(fd, parts, scratch, alloc_pinned, &ctx))
      break;
    if (!handle(parts, stream_recv)) break;
  }
}

// Refresh to a same-node client: no rows move.  The frame names the master
// version the client reads in place from now on (with the version buffer's IPC
// handle the first time this client sees it); the client releases the version
// it read before.  Returns false when the refresh must go as a copied frame;
// `*held`: the client now holds r.version.
bool ClientLib::ipc_reply(Channel &ch, uint32_t client_id, const RowBatchReply &r, bool *held) {
  *held = false;
  if (!ch.ipc_client[client_id] || r.version < 0 || r.num_rows == 0) return false;
  {
    std::lock_guard<std::mutex> lk(ch.ipc_mu);
    // A client that has shut down reads nothing more: the refresh is dropped
    // (and holds nothing: its SHUTDOWN released everything it held).
    if (ch.client_done[client_id]) return true;
  }
  IpcRefreshVersion rv{};
  rv.version = r.version;
  rv.num_rows = r.num_rows;
  bool first;
  {
    std::lock_guard<std::mutex> lk(ch.ipc_mu);  // (a NACK's resend erases from it on a reader thread)
    first = !ch.version_sent[client_id][r.table_id].count(r.version);
  }
  if (first) {
    if (!ipc_export(rv.handle, const_cast<float *>(r.device_rows), 1)) {
      // the runtime refused the export: this refresh goes as a copy
      std::lock_guard<std::mutex> lk(stats_mu_);
      stats_.nr_ipc_export_refused++;
      return false;
    }
    rv.has_handle = 1;
    {
      std::lock_guard<std::mutex> lk(ch.ipc_mu);
      ch.version_sent[client_id][r.table_id].insert(r.version);
    }
    if (ipc_log())
      std::cerr << "libgeeps ipc export version: server " << process_id_ << " ch " << ch.id << " client "
                << client_id << " table " << r.table_id << " version " << r.version << " rows " << r.num_rows
                << " at " << r.device_rows << ": " << ipc_describe(rv.handle) << "\n";
  }
  sc_read_row_batch_msg_t h{};
  h.cmd = READ_ROW_BATCH;
  h.server_id = r.server_id;
  h.data_age = r.data_age;
  h.self_clock = r.self_clock;
  h.table_id = r.table_id;
  GP_CHECK_MSG(send_to_client(ch, client_id, {Part{&h, sizeof h}, Part{nullptr, 0},
                                               Part{nullptr, 0}, Part{&rv, sizeof rv}}),
               "send to client " << client_id << " failed");
  *held = true;
  return true;
}


void ClientLib::send_to_server_chunked(Channel &ch, uint32_t s, const std::vector<Part> &parts,
                                       std::vector<std::unique_ptr<Event>> &events) {
  std::lock_guard<std::mutex> lk(*ch.server_send_mu[s]);
  GP_CHECK_MSG(!ch.server_shut[s], "send to server " << s << " after SHUTDOWN");
  GP_CHECK_MSG(send_frame_chunked(ch.server_fd[s], parts, kWireChunk, [&](size_t k) { events[k]->sync(); }),
               "send to server " << s << " failed");
}

void ClientLib::send_to_server(Channel &ch, uint32_t s, const std::vector<Part> &parts) {
  std::lock_guard<std::mutex> lk(*ch.server_send_mu[s]);
  GP_CHECK_MSG(!ch.server_shut[s], "send to server " << s << " after SHUTDOWN");
  GP_CHECK_MSG(send_frame(ch.server_fd[s], parts), "send to server " << s << " failed");
  if (parts.size() == 1 && parts[0].size == sizeof(cs_clock_msg_t) &&
      static_cast<const cs_clock_msg_t *>(parts[0].data)->cmd == SHUTDOWN)
    ch.server_shut[s] = 1;
}

// The reader thread releases a master version it no longer reads.  The last
// refresh can land after the app thread already sent SHUTDOWN (the server then
// reads nothing but kCmdReaderDone there, and its SHUTDOWN handling released
// every hold),
// so such a release is dropped, not sent.
void ClientLib::ack_to_server(Channel &ch, uint32_t s, const RefreshAckMsg &a) {
  std::lock_guard<std::mutex> lk(*ch.server_send_mu[s]);
  if (ch.server_shut[s]) return;
  GP_CHECK_MSG(send_frame(ch.server_fd[s], {Part{&a, sizeof a}}),
               "refresh ACK to server " << s << " failed");
}

void ClientLib::reader_done_to_server(Channel &ch, uint32_t s) {
  std::lock_guard<std::mutex> lk(*ch.server_send_mu[s]);
  cs_clock_msg_t h{};
  h.cmd = kCmdReaderDone;
  h.client_id = process_id_;
  GP_CHECK_MSG(send_frame(ch.server_fd[s], {Part{&h, sizeof h}}), "reader-done to server " << s << " failed");
}

void ClientLib::give_back(Channel &ch, uint32_t s, uint32_t table, int v) {
  if (s == process_id_) {
    ch.server->release(process_id_, table, v);
    return;
  }
  RefreshAckMsg a{};
  a.cmd = kCmdRefreshAck;
  a.client_id = process_id_;
  a.table_id = table;
  a.version = v;
  ack_to_server(ch, s, a);
}

void ClientLib::remote_shutdown_ack(uint32_t channel, uint32_t client_id) {
  if (client_id == process_id_) return;
  Channel &ch = *channels_[channel];
  cs_clock_msg_t h{};
  h.cmd = SHUTDOWN;
  h.client_id = process_id_;
  GP_CHECK_MSG(send_to_client(ch, client_id, {Part{&h, sizeof h}}),
               "shutdown ack to client " << client_id << " failed");
}

// The tablet server's reply to one client (read_row_batch_reply,
// server-encoder-decoder.cpp:228-250): in-process -> the client takes the
// master version in place (or copies it), same node -> the version by IPC,
// remote -> D2H into pinned memory and one frame on the client's socket.
bool ClientLib::remote_reply(uint32_t channel, uint32_t client_id, const RowBatchReply &r) {
  if (client_id == process_id_) {
    for (int v : recv_row_batch(channel, r.server_id, r.table_id, r.data_age, r.self_clock,
                                r.device_rows, r.num_rows, r.version))
      channels_[channel]->server->release(process_id_, r.table_id, v);
    return r.version >= 0;
  }
  Channel &ch = *channels_[channel];
  bool held = false;
  if (ipc_reply(ch, client_id, r, &held)) return held;
  const int fd = ch.client_fd[client_id];
  GP_CHECK_MSG(fd >= 0, "no connection to client " << client_id);
  const size_t floats = r.num_rows * ROW_DATA_SIZE;
  if (ch.reply_buf.size() < floats) ch.reply_buf.resize(floats);
  if (floats) copy_out_in_pieces(ch.reply_buf.data(), r.device_rows, floats * 4, *ch.svc_stream, ch.reply_events);
  sc_read_row_batch_msg_t h{};
  h.cmd = READ_ROW_BATCH;
  h.server_id = r.server_id;
  h.data_age = r.data_age;
  h.self_clock = r.self_clock;
  h.table_id = r.table_id;
  std::lock_guard<std::mutex> lk(*ch.client_send_mu[client_id]);
  GP_CHECK_MSG(send_frame_chunked(fd, {Part{&h, sizeof h}, Part{r.keys, r.num_rows * sizeof(RowKey)},
                                       Part{ch.reply_buf.data(), floats * 4}},
                                  kWireChunk, [&](size_t k) { ch.reply_events[k]->sync(); }),
               "send to client " << client_id << " failed");
  return false;
}

}  // namespace geeps
