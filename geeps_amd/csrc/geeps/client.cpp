// ClientLib — see client.hpp.  Reference: src/client/clientlib*.cpp.
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

namespace geeps {

ClientLib *client_lib = nullptr;

namespace {

double now_s() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

constexpr size_t kRowBytes = sizeof(RowData);
// How long a client retries connecting to a server that is not listening yet
// (processes start at different times); GEEPS_CONNECT_TIMEOUT_S overrides.
double connect_timeout_s() {
  const char *e = std::getenv("GEEPS_CONNECT_TIMEOUT_S");
  const double v = e ? std::atof(e) : 0.0;
  return v > 0 ? v : 300.0;
}
constexpr int kWaitWarnMs = 12000;  // the reference's 12 s timed_wait warnings

// GEEPS_IPC_LOG=1: one stderr line per IPC handle exported or mapped (which
// buffer, where, how large), on both sides, to audit buffer lifetimes.
bool ipc_log() {
  static const bool on = std::getenv("GEEPS_IPC_LOG") != nullptr;
  return on;
}

struct PinnedPool {
  std::vector<std::shared_ptr<PinnedArray<float>>> bufs;
  std::shared_ptr<PinnedArray<float>> get(size_t floats) {
    for (auto &b : bufs)
      if (b.use_count() == 1 && b->size() >= floats) return b;
    bufs.push_back(std::make_shared<PinnedArray<float>>(std::max<size_t>(floats, 1)));
    return bufs.back();
  }
};

}  // namespace

std::string ClientStats::to_json() const {
  std::ostringstream o;
  o << "{\"nr_read\": " << nr_read << ", \"nr_update\": " << nr_update
    << ", \"nr_clock\": " << nr_clock << ", \"nr_push\": " << nr_push
    << ", \"nr_refresh\": " << nr_refresh << ", \"nr_refresh_in_place\": " << nr_refresh_in_place
    << ", \"nr_refresh_staged\": " << nr_refresh_staged << ", \"nr_update_direct\": " << nr_update_direct
    << ", \"nr_read_direct\": " << nr_read_direct << ", \"nr_read_pin_deferred\": " << nr_read_pin_deferred
    << ", \"nr_read_direct_capped\": " << nr_read_direct_capped
    << ", \"nr_ipc_export_refused\": " << nr_ipc_export_refused << ", \"nr_ipc_nack_sent\": " << nr_ipc_nack_sent
    << ", \"nr_ipc_resent\": " << nr_ipc_resent << ", \"rows_host_tier\": " << rows_host_tier
    << ", \"nr_read_host\": " << nr_read_host << ", \"nr_update_host\": " << nr_update_host
    << ", \"nr_host_shared\": " << nr_host_shared << ", \"nr_host_share_refused\": " << nr_host_share_refused
    << ", \"rows_updated\": " << rows_updated
    << ", \"rows_read\": " << rows_read << ", \"bytes_pushed_remote\": " << bytes_pushed_remote
    << ", \"read_wait_time\": " << read_wait_time << ", \"read_time\": " << read_time
    << ", \"update_time\": " << update_time << ", \"push_time\": " << push_time
    << ", \"refresh_time\": " << refresh_time << "}";
  return o.str();
}

bool ChannelSink::read_row_batch_reply(uint32_t client_id, const RowBatchReply &r) {
  return lib_->remote_reply(channel_, client_id, r);
}

void ChannelSink::shutdown_ack(uint32_t client_id) { lib_->remote_shutdown_ack(channel_, client_id); }

// ---------------------------------------------------------------------------
// construction: servers, streams, sockets (clientlib.cpp:53-158)
// ---------------------------------------------------------------------------
ClientLib::ClientLib(uint32_t process_id, const GeePsConfig &config)
    : process_id_(process_id),
      config_(config),
      num_processes_((uint32_t)std::max<size_t>(1, config.host_list.size())),
      num_channels_(std::max(1u, config.num_comm_channels)) {
  GP_CHECK_MSG(process_id_ < num_processes_,
               "process_id " << process_id_ << " >= host_list.size() " << num_processes_);
  GP_CHECK(config_.num_tables > 0);
  GP_CHECK_MSG(config_.port_list.empty() || config_.port_list.size() >= num_processes_,
               "port_list must have one port per host");
  GP_CALL(gp_get_device(&device_));
  GP_CALL(gp_device_pci_bus_id(device_, pci_bus_id_, sizeof pci_bus_id_));
  // Same-node peers on another GPU: stage their buckets into local HBM before
  // the server's sum, and their refreshed shards into the local cache, by one
  // peer copy each (GEEPS_STAGE_PEER_UPDATES / GEEPS_STAGE_PEER_REFRESH: "1"
  // also on one GPU, which is how the cross-GPU path is tested on a one-GPU
  // box; "0" never: the kernels read the peer's HBM in place over xGMI).
  // Test hook (unset in production): GEEPS_TEST_READER_DELAY_US=D delays every
  // refresh a reader thread takes (a lagging client under SSP).
  auto mode = [](const char *name) {
    const char *v = std::getenv(name);
    return v && std::string(v) == "1" ? 1 : v && std::string(v) == "0" ? 0 : -1;
  };
  stage_updates_mode_ = mode("GEEPS_STAGE_PEER_UPDATES");
  stage_refresh_mode_ = mode("GEEPS_STAGE_PEER_REFRESH");
  const char *direct = std::getenv("GEEPS_DIRECT_OPLOG");
  direct_oplog_ = !(direct && std::string(direct) == "0");
  const char *direct_read = std::getenv("GEEPS_DIRECT_READ");
  direct_read_ = direct_read && std::string(direct_read) == "1";
  const char *delay = std::getenv("GEEPS_TEST_READER_DELAY_US");
  reader_delay_us_ = delay ? std::atoi(delay) : 0;
  if (const char *f = std::getenv("GEEPS_TEST_IPC_FAULT"))
    ipc_fault_ = std::string(f) == "tag" ? 1 : std::string(f) == "refuse" ? 2 : 0;
  // Same-node peers exchange rows device to device through IPC-mapped HBM
  // (xGMI between GPUs); GEEPS_TRANSPORT=tcp forces the socket data path.
  const char *transport = std::getenv("GEEPS_TRANSPORT");
  const bool allow_ipc = !(transport && std::string(transport) == "tcp");
  auto norm = [](const std::string &h) {
    return (h == "localhost" || h == "local" || h == "127.0.0.1") ? std::string("127.0.0.1") : h;
  };
  same_node_.assign(num_processes_, false);
  for (uint32_t s = 0; s < num_processes_; ++s)
    same_node_[s] = allow_ipc && num_processes_ > 1 &&
                    norm(config_.host_list[s]) == norm(config_.host_list[process_id_]);
  const char *share = std::getenv("GEEPS_HOST_SHARE");
  host_share_ = config_.pinned_cpu_memory != 0 && !(share && std::string(share) == "0");
  bool any_peer = false;
  for (uint32_t s = 0; s < num_processes_; ++s) any_peer |= ipc_to(s);
  host_share_ = host_share_ && any_peer;
  channels_.resize(num_channels_);
  for (uint32_t c = 0; c < num_channels_; ++c) {
    auto ch = std::make_unique<Channel>();
    ch->id = c;
    ch->tables.resize(config_.num_tables);
    ch->stream = std::make_unique<Stream>();
    ch->svc_stream = std::make_unique<Stream>();
    ch->sink = std::make_unique<ChannelSink>(this, c);
    ch->server = std::make_unique<TabletServer>(process_id_, c, num_processes_,
                                                config_.num_tables, ch->sink.get(), device_,
                                                ch->svc_stream->get());
    ch->server_fd.assign(num_processes_, -1);
    for (uint32_t s = 0; s < num_processes_; ++s)
      ch->server_send_mu.push_back(std::make_unique<std::mutex>());
    ch->server_shut.assign(num_processes_, 0);
    ch->client_fd.assign(num_processes_, -1);
    for (uint32_t s = 0; s < num_processes_; ++s)
      ch->client_send_mu.push_back(std::make_unique<std::mutex>());
    ch->ipc_oplogs.resize(num_processes_);
    ch->host_oplogs.resize(num_processes_);
    ch->host_share_off.assign(num_processes_, 0);
    ch->ipc_client.assign(num_processes_, 0);
    ch->other_gpu.assign(num_processes_, 0);
    ch->stage_from.assign(num_processes_, 0);
    ch->stage_refresh_from.assign(num_processes_, 0);
    ch->version_sent.assign(num_processes_, std::vector<std::set<int>>(config_.num_tables));
    ch->client_done.assign(num_processes_, 0);
    channels_[c] = std::move(ch);
  }
  start_network();
}

ClientLib::~ClientLib() { shutdown(); }

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
            GP_CALL(gp_ipc_close_handle(old->second));
            mapped.erase(old);
          }
          void *p = nullptr;
          ok = gp_ipc_open_handle(&p, ref.handle) == GP_OK;
          if (ok) {
            mapped[ref.buffer_id] = p;
            if (ipc_log())
              std::cerr << "libgeeps ipc map oplog: server " << process_id_ << " ch " << ch.id << " client "
                        << client_id << " buffer " << ref.buffer_id << " -> " << p << "\n";
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

namespace {
// Rows bound for a socket leave the GPU in pieces of this size, each sent as
// soon as its copy lands (send_frame_chunked), so the D2H of a large slice
// overlaps the send instead of preceding it.
constexpr size_t kWireChunk = 16u << 20;

// The device-to-host copy of `bytes` from `src` into pinned `dst` on `st`, an
// event recorded after each kWireChunk piece.
void copy_out_in_pieces(void *dst, const void *src, size_t bytes, const Stream &st,
                        std::vector<std::unique_ptr<Event>> &events) {
  const size_t pieces = (bytes + kWireChunk - 1) / kWireChunk;
  while (events.size() < pieces) events.push_back(std::make_unique<Event>());
  for (size_t k = 0; k < pieces; ++k) {
    const size_t off = k * kWireChunk, len = std::min(kWireChunk, bytes - off);
    GP_CALL(gp_memcpy_async(static_cast<char *>(dst) + off, static_cast<const char *>(src) + off, len, st.get()));
    events[k]->record(st);
  }
}
}  // namespace

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
                      << rv.num_rows << " -> " << ptr << "\n";
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
                << " at " << r.device_rows << "\n";
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

// ---------------------------------------------------------------------------
// virtual iteration (clientlib-viter.cpp)
// ---------------------------------------------------------------------------
int ClientLib::virtual_op(OpInfo &&op) {
  GP_CHECK_MSG(!finished_vi_, "virtual op after FinishVirtualIteration");
  opseq_.push_back(std::move(op));
  return (int)opseq_.size() - 1;
}

uint32_t ClientLib::channel_of(uint32_t table_id, row_idx_t row) const {
  return (uint32_t)(row / rows_per_channel_[table_id]);  // clientlib.cpp:216-219
}

// vi_create_local_storage (clientlib-viter.cpp:160-490), reduced to what it
// leaves used of ngr_capacity before the param cache: the local key batches
// that are fetched or kept go to GPU memory when they fit beside a thread
// cache of twice the peak rows in use at once (the op buffers of READ /
// PRE_WRITE ops, counted from an op to its post-step; GPU local storage is not
// counted in the peak), and the thread cache takes twice that peak.  libgeeps
// keeps every local batch in HBM (no CPU local storage): when the fetched /
// kept batches do not fit, the reference would place some in CPU memory,
// which it allows below mm_warning_level 2 -- here that is a warning.
size_t ClientLib::reference_ngr_used(size_t ngr_capacity) {
  struct Batch {
    size_t rows = 0;
    bool fetchkeep = false;
  };
  std::map<std::pair<uint64_t, row_idx_t>, Batch> local;  // (table, first row)
  auto key_of = [](const OpInfo &op) { return std::make_pair((uint64_t)op.table, op.rows[0]); };
  for (auto &op : opseq_) {
    if (op.local && op.type == OpInfo::READ && !op.rows.empty()) {
      Batch &b = local[key_of(op)];
      b.rows = op.rows.size();
      b.fetchkeep = b.fetchkeep || op.fetch;
    }
    if (op.type == OpInfo::POST_READ && op.local && op.keep) {
      const OpInfo &pre = opseq_[op.prestep_handle];
      if (!pre.rows.empty()) local[key_of(pre)].fetchkeep = true;
    }
  }
  size_t fetchkeep_rows = 0;
  for (auto &kv : local) fetchkeep_rows += kv.second.fetchkeep ? kv.second.rows : 0;
  // the peak of op rows in use at once, local batches in GPU memory excluded
  auto peak_rows = [&](bool fetchkeep_in_gpu) {
    size_t now = 0, peak = 0;
    auto counted = [&](const OpInfo &op) {
      return !(op.local && !op.rows.empty() && fetchkeep_in_gpu && local[key_of(op)].fetchkeep);
    };
    for (auto &op : opseq_) {
      if ((op.type == OpInfo::READ || op.type == OpInfo::PRE_WRITE) && counted(op)) {
        now += op.rows.size();
        peak = std::max(peak, now);
      } else if (op.type == OpInfo::POST_READ || op.type == OpInfo::WRITE) {
        const OpInfo &pre = opseq_[op.prestep_handle];
        if (counted(pre)) now -= std::min(now, pre.rows.size());
      }
    }
    return peak;
  };
  const size_t peak0 = peak_rows(false);
  GP_CHECK_MSG(ngr_capacity / 2 >= peak0, "gpu_memory_capacity holds " << ngr_capacity << " RowData rows, "
               "less than twice the peak " << peak0 << " rows of ops in use at once (the thread cache, "
               "clientlib-viter.cpp:338)");
  size_t used = fetchkeep_rows, peak = peak0;
  if (fetchkeep_rows + 2 * peak0 <= ngr_capacity) {
    peak = peak_rows(true);
  } else if (fetchkeep_rows) {
    GP_CHECK_MSG(config_.mm_warning_level < 2,
                 "local storage (" << fetchkeep_rows << " rows fetched or kept) does not fit gpu_memory_capacity "
                 "beside the thread cache, and mm_warning_level 2 keeps all local data in GPU memory");
    std::cerr << "libgeeps WARNING: local storage past gpu_memory_capacity stays in HBM (no CPU local "
                 "storage tier)\n";
  }
  size_t thread_cache = 2 * peak;
  const size_t left = ngr_capacity > used ? ngr_capacity - used : 0;
  if (thread_cache > left) {
    GP_CHECK_MSG(config_.mm_warning_level < 1, "not enough space for double buffering (thread cache of "
                 << thread_cache << " rows, " << left << " left; clientlib-viter.cpp:482-487)");
    std::cerr << "*** WARNING: not enough space for double buffering\n";
    thread_cache = left;
  }
  return used + thread_cache;
}

void ClientLib::finish_virtual_iteration() {
  GP_CHECK(!finished_vi_);
  finished_vi_ = true;
  const uint32_t T = config_.num_tables;

  // Post-steps inherit their pre-step's table and locality (vi_thread_finalize).
  for (auto &op : opseq_) {
    if (op.type == OpInfo::WRITE || op.type == OpInfo::POST_READ) {
      GP_CHECK(op.prestep_handle >= 0 && (size_t)op.prestep_handle < opseq_.size());
      const OpInfo &pre = opseq_[op.prestep_handle];
      GP_CHECK(pre.type == (op.type == OpInfo::WRITE ? OpInfo::PRE_WRITE : OpInfo::READ));
      op.local = pre.local;
      op.table_id = pre.table_id;
    } else if ((op.type == OpInfo::READ || op.type == OpInfo::PRE_WRITE) && !op.local) {
      GP_CHECK_MSG(op.table < T, "table " << op.table << " >= num_tables " << T);
      op.table_id = (uint32_t)op.table;
    }
  }
  for (auto &op : opseq_)
    if ((op.type == OpInfo::WRITE || op.type == OpInfo::POST_READ) && !op.local)
      op.table_id = opseq_[op.prestep_handle].table_id;

  // Last write of each table, among the ops up to the last CLOCK.
  std::vector<bool> seen(T, false);
  bool clock_seen = false;
  for (size_t i = opseq_.size(); i-- > 0;) {
    OpInfo &op = opseq_[i];
    if (op.type == OpInfo::CLOCK) clock_seen = true;
    if (!clock_seen) continue;
    if (!op.local && op.type == OpInfo::WRITE && !seen[op.table_id]) {
      seen[op.table_id] = true;
      op.table_last_write = true;
    }
  }
  for (uint32_t t = 0; t < T; ++t) GP_CHECK_MSG(seen[t], "No one writes table " << t);

  // Oplog entries per cache row: 1, or slack + 1 with read-my-writes
  // (vi_decide_param_cache, clientlib-viter.cpp:507-517); used for planning
  // (and the placement below), the pool grows on demand.
  iter_t max_slack = 0;
  for (auto &op : opseq_)
    if (!op.local && op.type == OpInfo::READ) max_slack = std::max(max_slack, op.slack);
  const size_t entries = config_.read_my_writes ? (size_t)max_slack + 1 : 1;

  // Param cache rows in first-access order per table, each new key batch
  // placed as vi_decide_param_cache places it (clientlib-viter.cpp:520-568):
  // in HBM while (HBM rows + batch) x (1 + oplog entries) fits what
  // gpu_memory_capacity leaves after local storage and the thread cache
  // (counted in RowData rows, ngr_capacity = capacity / sizeof(RowData),
  // :179), else in the host tier.  A later op's keys keep their batch's place.
  const size_t ngr_capacity = config_.gpu_memory_capacity / sizeof(RowData);
  const size_t ngr_used = reference_ngr_used(ngr_capacity);
  const size_t ngr_param = ngr_capacity > ngr_used ? ngr_capacity - ngr_used : 0;
  const size_t entries_per_row = 1 + entries;
  size_t gpu_rows = 0;
  std::vector<std::vector<row_idx_t>> keys(T);
  std::vector<std::unordered_map<row_idx_t, bool>> on_gpu(T);
  for (auto &op : opseq_) {
    if (op.local || (op.type != OpInfo::READ && op.type != OpInfo::PRE_WRITE) || op.rows.empty())
      continue;
    auto &kn = on_gpu[op.table_id];
    auto first = kn.find(op.rows[0]);
    if (first == kn.end()) {
      // a new key batch: (gpu rows + batch) x entries_per_row <= capacity left
      const size_t n = op.rows.size();
      const bool gpu = n <= ngr_param / entries_per_row && gpu_rows <= ngr_param / entries_per_row - n;
      if (!gpu)
        GP_CHECK_MSG(config_.mm_warning_level < 3,
                     "a key batch of " << n << " rows of table " << op.table_id << " does not fit "
                     "gpu_memory_capacity (" << config_.gpu_memory_capacity << " B: " << ngr_capacity
                     << " RowData rows, " << ngr_used << " for local storage and the thread cache, "
                     << gpu_rows << " x " << entries_per_row << " for the param cache so far), and "
                     "mm_warning_level 3 keeps all parameter cache in GPU memory "
                     "(clientlib-viter.cpp:551-552)");
      for (row_idx_t r : op.rows) {
        GP_CHECK_MSG(!kn.count(r), "row " << r << " of a new key batch already cached");
        kn[r] = gpu;
        keys[op.table_id].push_back(r);
      }
      if (gpu) gpu_rows += n;
      op.cpu = !gpu;
    } else {
      op.cpu = !first->second;
      for (row_idx_t r : op.rows) {
        auto it = kn.find(r);
        GP_CHECK_MSG(it != kn.end(), "row " << r << " mixes new and cached keys in one op");
        GP_CHECK_MSG(it->second == first->second,
                     "row " << r << " of an op lies in another param-cache tier than the op's first row");
      }
    }
  }
  // Post-steps take their pre-step's placement.
  for (auto &op : opseq_)
    if ((op.type == OpInfo::WRITE || op.type == OpInfo::POST_READ) && !op.local)
      op.cpu = opseq_[op.prestep_handle].cpu;
  rows_per_channel_.assign(T, 1);
  for (uint32_t t = 0; t < T; ++t)
    rows_per_channel_[t] = std::max<size_t>(1, (keys[t].size() + num_channels_ - 1) / num_channels_);

  size_t planned = 0;
  for (auto &chp : channels_) {
    Channel &ch = *chp;
    for (uint32_t t = 0; t < T; ++t) {
      ParamCache &pc = ch.tables[t];
      HostTier &cpu = pc.cpu;
      // each tier's rows in first-access order (vi_process_channel_table_
      // finalize runs once per tier over its key list, clientlib-viter.cpp:624-662)
      for (row_idx_t r : keys[t]) {
        if (channel_of(t, r) != ch.id) continue;
        if (on_gpu[t].at(r)) {
          pc.index[r] = pc.num_rows++;
          pc.row_keys->emplace_back(t, r);
        } else {
          cpu.index[r] = cpu.num_rows++;
          cpu.row_keys.emplace_back(t, r);
        }
      }
      if (cpu.num_rows) {
        cpu.data = std::make_unique<HostBuf>(cpu.num_rows * ROW_DATA_SIZE, config_.pinned_cpu_memory != 0);
        cpu.data->zero();  // zerofy_data_cpu
        cpu.server_row_start.resize(num_processes_);
        cpu.server_num_rows.resize(num_processes_);
        const size_t div = cpu.num_rows / num_processes_, res = cpu.num_rows % num_processes_;
        for (size_t i = 0; i < num_processes_; ++i) {
          cpu.server_row_start[i] = div * i + std::min(i, res);
          cpu.server_num_rows[i] = div + (i < res ? 1 : 0);
        }
        std::lock_guard<std::mutex> lk(stats_mu_);
        stats_.rows_host_tier += cpu.num_rows;
      }
      pc.server_row_start.resize(num_processes_);
      pc.server_num_rows.resize(num_processes_);
      {
        const size_t div = pc.num_rows / num_processes_, res = pc.num_rows % num_processes_;
        for (size_t i = 0; i < num_processes_; ++i) {
          pc.server_row_start[i] = div * i + std::min(i, res);
          pc.server_num_rows[i] = div + (i < res ? 1 : 0);
        }
      }
      // The cache's own rows are needed only for refreshes that arrive as
      // copies (socket peers, staged peers on another GPU, read-my-writes,
      // which also scatters into it).  When every server's shard will be read
      // in place, it is never touched (a Read waits for every server's first
      // refresh) and is not allocated.  Without read-my-writes each copied
      // shard gets a buffer of its own, which refreshes replace by a swap
      // (shard_buf); with it, the one flat `data` the Updates scatter into.
      auto copied = [&](uint32_t s) { return s != process_id_ && (!ipc_to(s) || ch.stage_refresh_from[s]); };
      bool copies = false;
      for (uint32_t s = 0; s < num_processes_; ++s) copies = copies || copied(s);
      if (config_.read_my_writes) {
        pc.data.resize(pc.num_rows * ROW_DATA_SIZE);
        if (pc.num_rows) GP_CALL(gp_zero(pc.data.data(), pc.data.size(), ch.stream->get()));
        planned += pc.data.bytes();
      } else if (copies) {
        pc.shard_buf.resize(num_processes_);
        for (uint32_t s = 0; s < num_processes_; ++s) {
          if (!copied(s) || pc.server_num_rows[s] == 0) continue;
          pc.shard_buf[s].resize(pc.server_num_rows[s] * ROW_DATA_SIZE);
          GP_CALL(gp_zero(pc.shard_buf[s].data(), pc.shard_buf[s].size(), ch.stream->get()));
          planned += pc.shard_buf[s].bytes();
        }
      }
      planned += pc.num_rows * kRowBytes * entries;
      // the server's staging buckets: one per pending bucket of a peer on
      // another GPU (its slice peer-copied in) or of a remote client (its
      // socket rows copied in), at most kMaxPendingBuckets (the queue is
      // applied when it reaches that many)
      size_t staged_peers = 0;
      for (uint32_t s = 0; s < num_processes_; ++s)
        staged_peers += (ch.stage_from[s] || (s != process_id_ && !ipc_to(s))) ? 1 : 0;
      // + this process's server's master versions of the shard: two (the
      // current one and the next, built beside it while clients read it in
      // place); a lagging reader can make it up to clients + 2 (server.hpp)
      planned += pc.server_num_rows[process_id_] * kRowBytes *
                 (std::min<size_t>(staged_peers, TabletServer::kMaxPendingBuckets) + 2);
      // + a landing buffer per socket server (its reader streams a refresh's
      // rows into HBM as they arrive) and per staged same-node server (its
      // reader peer-copies a refresh there outside the channel lock,
      // client_reader): that server's shard
      for (uint32_t s = 0; s < num_processes_; ++s)
        if (s != process_id_ && (!ipc_to(s) || ch.stage_refresh_from[s])) planned += pc.server_num_rows[s] * kRowBytes;
      pc.per_server_data_age.assign(num_processes_, INITIAL_DATA_AGE);
      pc.live_ver.assign(num_processes_, -1);
      pc.live_ptr.assign(num_processes_, nullptr);
      pc.server_versions.resize(num_processes_);
      pc.pins.assign(num_processes_, {});
      pc.deferred.assign(num_processes_, {});
      pc.read_events.assign(num_processes_, {});
      pc.server_clock.assign(num_processes_, INITIAL_DATA_AGE);
      if (cpu.num_rows) {
        // every server's frame keys: its host-tier keys, then its HBM-tier keys
        // (clientlib-data.cpp:487-509: the CPU part first)
        pc.frame_keys.resize(num_processes_);
        for (uint32_t s = 0; s < num_processes_; ++s) {
          auto k = std::make_shared<std::vector<RowKey>>();
          k->insert(k->end(), cpu.row_keys.begin() + cpu.server_row_start[s],
                    cpu.row_keys.begin() + cpu.server_row_start[s] + cpu.server_num_rows[s]);
          k->insert(k->end(), pc.row_keys->begin() + pc.server_row_start[s],
                    pc.row_keys->begin() + pc.server_row_start[s] + pc.server_num_rows[s]);
          pc.frame_keys[s] = k;
        }
        // the server stages every batch with a host part (one bucket each)
        planned += (pc.server_num_rows[process_id_] + cpu.server_num_rows[process_id_]) * kRowBytes *
                   TabletServer::kMaxPendingBuckets;
      }
      rebuild_segments(pc);
    }
    ch.stream->sync();
  }
  for (auto &chp : channels_)
    for (uint32_t t = 0; t < T; ++t)
      GP_CHECK_MSG(chp->tables[t].num_rows + chp->tables[t].cpu.num_rows <= rows_per_channel_[t] ||
                       num_channels_ == 1,
                   "channel " << chp->id << " of table " << t << " holds rows past its range");

  // Op buffers, DoubleIndex, local storage.
  for (auto &op : opseq_) {
    if (op.type != OpInfo::READ && op.type != OpInfo::PRE_WRITE) continue;
    if (op.local) {
      auto &slot = local_storage_[op.rows];
      if (!slot) {
        slot = std::make_unique<DeviceArray<float>>(std::max<size_t>(1, op.rows.size()) * ROW_DATA_SIZE);
        GP_CALL(gp_zero(slot->data(), slot->size(), channels_[0]->stream->get()));
        planned += slot->bytes();
      }
      op.local_ptr = slot->data();
      continue;
    }
    op.buffer.resize(std::max<size_t>(1, op.rows.size()) * ROW_DATA_SIZE);
    GP_CALL(gp_zero(op.buffer.data(), op.buffer.size(), channels_[0]->stream->get()));
    planned += op.buffer.bytes();
    if (op.cpu && cpu_buffer_.size() < op.rows.size() * ROW_DATA_SIZE)
      cpu_buffer_.resize(op.rows.size() * ROW_DATA_SIZE);  // max_nr_each_access rows (clientlib-viter.cpp:444-447)
    // the device DoubleIndex, and an update or read op's row plans (a sorted copy)
    planned += op.rows.size() * sizeof(gp_double_index) *
               (op.type == OpInfo::PRE_WRITE || op.type == OpInfo::READ ? 2 : 1);
    create_double_index(op);
  }
  GP_CALL(gp_device_synchronize());
  decide_fused_init();
  if (planned > config_.gpu_memory_capacity && config_.mm_warning_level >= 1) {
    // The param cache's rows were placed by the reference's own model above
    // (rows past the capacity went to the host tier).  What that model does
    // not count is what libgeeps keeps in HBM beyond it: the tablet server's
    // master versions and staging buckets (the reference's server is CPU
    // memory), the op buffers and plans.
    std::cerr << "libgeeps WARNING: planned HBM use " << planned << " B (param cache, oplogs, op buffers, "
              << "and this process's tablet-server shards and staging buffers) exceeds gpu_memory_capacity "
              << config_.gpu_memory_capacity << " B\n";
  }
}

// Per (channel, table): do the update ops of one clock (the WRITEs before the
// first CLOCK op) write every oplog row exactly once, unguarded?  Then, after
// StartIterations (when the op order is enforced), each op may write its rows as
// 0.0f + x instead of zerofying the whole oplog and adding: bit-identical, one
// pass fewer over the oplog (see gp_scatter_init_rows).
void ClientLib::decide_fused_init() {
  clock_handle_ = -1;
  for (size_t i = 0; i < opseq_.size(); ++i)
    if (opseq_[i].type == OpInfo::CLOCK) {
      clock_handle_ = (int)i;
      break;
    }
  const size_t end = clock_handle_ < 0 ? opseq_.size() : (size_t)clock_handle_;
  for (auto &chp : channels_) {
    Channel &ch = *chp;
    ch.init_ok.assign(config_.num_tables, false);
    if (clock_handle_ < 0) continue;
    for (uint32_t t = 0; t < config_.num_tables; ++t) {
      const ParamCache &pc = ch.tables[t];
      std::vector<uint8_t> seen(pc.num_rows, 0);
      size_t covered = 0, writers = 0;
      bool ok = pc.num_rows > 0;
      for (size_t i = 0; i < end && ok; ++i) {
        const OpInfo &w = opseq_[i];
        if (w.type != OpInfo::WRITE || w.local || w.table_id != t || w.cpu) continue;  // (host-tier ops: its own oplog)
        const OpInfo &pre = opseq_[w.prestep_handle];
        bool here = false;
        if (pre.num_vals_limit < pre.rows.size() * ROW_DATA_SIZE) ok = false;
        // the op's id1 set in this channel is the contiguous range checked in
        // create_double_index; recover it from the row ids
        for (row_idx_t r : pre.rows) {
          if (channel_of(t, r) != ch.id) continue;
          const size_t id1 = pc.index.at(r);
          if (seen[id1]++) ok = false;
          ++covered;
          here = true;
        }
        writers += here;
      }
      // Read-my-writes re-applies a refresh's pending oplogs, the current
      // clock's included (recv_row_batch): its rows must be zero until an op
      // writes them, as after the reference's zerofy (clientlib-data.cpp:
      // 356-371).  With ONE update op per clock in this (channel, table) the
      // oplog is created and fully written inside that Update, under the
      // channel lock a refresh takes too (and synced before it is released),
      // so no refresh sees it unwritten: the fused init stays.  With several,
      // a refresh between two of them would: zeroed oplog.
      ch.init_ok[t] = ok && covered == pc.num_rows && (!config_.read_my_writes || writers == 1);
    }
  }
  // Direct oplog: an update op whose rows are one channel's cache rows in
  // order, in a (channel, table) whose clock writes every oplog row once.
  // The app's buffer then IS the oplog slice: the fused init's copy
  // (0.0f + x) disappears.  The slice holds x instead of 0.0f + x, which
  // differs only for -0.0 (and a signalling NaN's quiet bit); the server's
  // master starts at +0.0 and a sum is -0.0 only when both addends are, so
  // every master row, partial sum and refresh is bit-identical.
  for (size_t i = 0; i < end; ++i) {
    OpInfo &w = opseq_[i];
    if (w.type != OpInfo::WRITE || w.local) continue;
    OpInfo &pre = opseq_[w.prestep_handle];
    // (not with read-my-writes: the app would write the oplog between
    // PreUpdate and Update, outside the channel lock a refresh's re-apply of
    // that oplog takes)
    pre.direct = direct_oplog_ && pre.direct_channel >= 0 && !pre.rows.empty() &&
                 channels_[pre.direct_channel]->init_ok[pre.table_id] && !config_.read_my_writes;
  }
}

// One DoubleIndex per op, grouped by channel, each channel's id1 range equal
// to its row count (vi_create_double_index, clientlib-viter.cpp:817-883: the
// CHECK_EQ at :871-873).  Like the reference this admits a repeated row when
// the range still matches (cache rows {0, 0, 2}); the row plans add its
// occurrences in op order, as the reference's CPU twin does (row-op-util.hpp:
// 121-139; its GPU kernel races on such a row).
void ClientLib::create_double_index(OpInfo &op) {
  std::vector<std::vector<gp_double_index>> per(num_channels_);
  for (size_t j = 0; j < op.rows.size(); ++j) {
    const uint32_t c = channel_of(op.table_id, op.rows[j]);
    GP_CHECK_LT(c, num_channels_);
    ParamCache &pc = channels_[c]->tables[op.table_id];
    auto &index = op.cpu ? pc.cpu.index : pc.index;  // the op's tier
    auto it = index.find(op.rows[j]);
    GP_CHECK_MSG(it != index.end(), "row " << op.rows[j] << " not in the param cache");
    per[c].push_back(gp_double_index{j, it->second});
  }
  std::vector<gp_double_index> flat;
  flat.reserve(op.rows.size());
  op.ch_start.assign(num_channels_, 0);
  op.ch_size.assign(num_channels_, 0);
  for (uint32_t c = 0; c < num_channels_; ++c) {
    op.ch_start[c] = flat.size();
    op.ch_size[c] = per[c].size();
    if (!per[c].empty()) {
      uint64_t lo = per[c][0].id1, hi = lo;
      std::unordered_set<uint64_t> ids;
      for (auto &d : per[c]) {
        lo = std::min<uint64_t>(lo, d.id1);
        hi = std::max<uint64_t>(hi, d.id1);
        ids.insert(d.id1);
      }
      op.repeats = op.repeats || ids.size() != per[c].size();
      GP_CHECK_EQ(hi - lo + 1, (uint64_t)per[c].size());
    }
    flat.insert(flat.end(), per[c].begin(), per[c].end());
  }
  // The update ops' oplog accumulate runs through a row plan per channel: the
  // same rows visited in cache-row order (bit-identical: a repeated id1 gets
  // its adds in op order through the plan's repeat layers), so the scatter's
  // read-modify-write side walks the oplog in order.
  // The read ops' gather runs through a gather plan per channel: its dense
  // runs (first-access order makes an op's rows one run per channel) are
  // copied by the phase-separated kernels, which hold their rate on every
  // allocation.
  if (op.cpu) {
    // a host-tier op: its index stays in host memory (the reference's
    // row_index_cpu, clientlib-viter.cpp:853-876); no device index or plans
    op.host_index = std::move(flat);
    op.direct_channel = -1;
    return;
  }
  if (op.type == OpInfo::PRE_WRITE || op.type == OpInfo::READ) {
    op.direct_channel = -1;
    for (uint32_t c = 0; c < num_channels_; ++c) {
      if (per[c].size() != op.rows.size() || op.rows.empty()) continue;
      bool run = true;
      for (size_t j = 0; j < per[c].size() && run; ++j)
        run = per[c][j].id0 == j && per[c][j].id1 == per[c][0].id1 + j;
      if (run) {
        op.direct_channel = (int)c;
        op.direct_lo = per[c][0].id1;
      }
    }
  }
  if (op.type == OpInfo::PRE_WRITE || op.type == OpInfo::READ) {
    op.plans.resize(num_channels_);
    for (uint32_t c = 0; c < num_channels_; ++c)
      if (!per[c].empty())
        op.plans[c] = std::make_unique<RowPlan>(per[c].data(), per[c].size(), ROW_DATA_SIZE,
                                                op.num_vals_limit, op.type == OpInfo::READ);
  }
  op.index.resize(std::max<size_t>(1, flat.size()));
  if (!flat.empty())
    GP_CALL(gp_memcpy_async(op.index.data(), flat.data(), flat.size() * sizeof(gp_double_index),
                            channels_[0]->stream->get()));
  channels_[0]->stream->sync();
}

void ClientLib::start_iterations() {
  GP_CHECK_MSG(finished_vi_, "StartIterations before FinishVirtualIteration");
  started_ = true;
  last_handle_ = -1;
}

void ClientLib::check_handle(int handle) {
  GP_CHECK(handle >= 0 && (size_t)handle < opseq_.size());
  if (started_) {
    GP_CHECK_MSG(handle == last_handle_ + 1,
                 "handle mismatch: " << handle << " after " << last_handle_);
    last_handle_ = handle;
  }
}

// ---------------------------------------------------------------------------
// Read / PostRead (clientlib.cpp:349-473; clientlib-data.cpp:191-278)
// ---------------------------------------------------------------------------
bool ClientLib::read_batch(RowData **buffer, int handle) {
  check_handle(handle);
  OpInfo &op = opseq_[handle];
  GP_CHECK(op.type == OpInfo::READ);
  GP_CHECK_MSG(!op.in_use, "Read of handle " << handle << " before its PostRead");
  if (op.local) {
    *buffer = reinterpret_cast<RowData *>(op.local_ptr);
    op.in_use = true;
    return true;
  }
  if (op.cpu) {
    read_batch_host(op);
    *buffer = reinterpret_cast<RowData *>(op.buffer.data());
    op.in_use = true;
    return true;
  }
  const double t0 = now_s();
  const iter_t need = iteration_ - op.slack - 1;
  double waited = 0;
  float *direct = nullptr;
  bool capped = false;
  for (auto &chp : channels_) {
    Channel &ch = *chp;
    ParamCache &pc = ch.tables[op.table_id];
    std::unique_lock<std::mutex> lk(ch.mu);
    const double w0 = now_s();
    while (pc.data_age < need) {
      if (!ch.cv.wait_for(lk, std::chrono::milliseconds(kWaitWarnMs),
                          [&] { return pc.data_age >= need; }) &&
          ch.id == 0) {
        std::cerr << "machine " << process_id_ << " wait time out! Need: " << need
                  << " Data age: " << pc.data_age << std::endl;
      }
    }
    waited += now_s() - w0;
    // (an op whose last row straddles num_vals_limit gathers: its buffer holds
    // zeros past the limit, which the master's rows do not)
    if (direct_read_ && started_ && op.direct_channel == (int)ch.id &&
        op.num_vals_limit >= op.rows.size() * ROW_DATA_SIZE) {
      // Direct read: the op's rows are one server's shard rows in order and
      // that shard is read in place, so the buffer is the master version's own
      // rows.  The version stays pinned (not given back, so the server never
      // writes it) until PostRead.
      const size_t lo = op.direct_lo, n = op.rows.size();
      for (uint32_t s = 0; s < num_processes_; ++s) {
        const size_t first = pc.server_row_start[s];
        if (lo < first || lo + n > first + pc.server_num_rows[s] || pc.live_ver[s] < 0) continue;
        // at most one deferred (replaced but pinned) version per server: a
        // second one could leave the server's version cap waiting on this app
        // thread's PostRead while the thread waits in a Read
        if (!pc.deferred[s].empty() && !pc.pins[s].count(pc.live_ver[s])) {
          capped = true;
          break;
        }
        direct = const_cast<float *>(pc.live_ptr[s]) + (lo - first) * ROW_DATA_SIZE;
        op.pin_server = (int)s;
        op.pin_version = pc.live_ver[s];
        ++pc.pins[s][op.pin_version];
        break;
      }
      if (direct) continue;
    }
    // assign_rows_to_double_index_gpu (clientlib-data.cpp:254-278) through the
    // op's gather plan for this channel (its index, offset 0, num_vals_limit)
    float *const y = reinterpret_cast<float *>(op.buffer.data());
    if (op.ch_size[ch.id] && pc.segmented)
      GP_CALL(gp_gather_rows_segmented_planned(y, &pc.segs, op.plans[ch.id]->get(), ch.stream->get()));
    else if (op.ch_size[ch.id])
      GP_CALL(gp_gather_rows_planned(y, pc.data.data(), op.plans[ch.id]->get(), ch.stream->get()));
    ch.stream->sync();
  }
  *buffer = reinterpret_cast<RowData *>(direct ? direct : op.buffer.data());
  op.in_use = true;
  std::lock_guard<std::mutex> lk(stats_mu_);
  stats_.nr_read++;
  if (direct) stats_.nr_read_direct++;
  if (capped) stats_.nr_read_direct_capped++;
  stats_.rows_read += op.rows.size();
  stats_.read_wait_time += waited;
  stats_.read_time += now_s() - t0;
  return true;
}

namespace {
// A host-tier op's rows cross PCIe in pieces of this many rows (16 MiB), so
// that the CPU's gather or scatter-add of one piece overlaps the copy of the
// next.
constexpr size_t kHostPieceRows = (16u << 20) / kRowBytes;

// The entries [lo, hi) of one channel's host DoubleIndex whose op-buffer row
// (id0) lies in [r0, r1): create_double_index lists them in op-row order.
std::pair<size_t, size_t> entries_in(const gp_double_index *idx, size_t n, size_t r0, size_t r1) {
  auto below = [](const gp_double_index &d, size_t r) { return d.id0 < r; };
  const gp_double_index *lo = std::lower_bound(idx, idx + n, r0, below);
  const gp_double_index *hi = std::lower_bound(lo, idx + n, r1, below);
  return {(size_t)(lo - idx), (size_t)(hi - idx)};
}
}  // namespace

// A host-tier op's Read: per channel, wait for the data age and gather the
// op's rows from the host cache into the pinned host buffer (read_batch_cpu,
// assign_rows_to_double_index_cpu: clientlib-data.cpp:280-302); then the
// host-to-device copy of num_vals_limit floats into the op buffer in HBM
// (read_row_batch_param_cache, :233-250).  The last channel gathers piece by
// piece, and each piece's copy starts as soon as it is gathered (every
// channel holds its lock for the whole of its gather, as in the reference).
void ClientLib::read_batch_host(OpInfo &op) {
  const double t0 = now_s();
  const iter_t need = iteration_ - op.slack - 1;
  double waited = 0;
  for (auto &chp : channels_) {
    Channel &ch = *chp;
    ParamCache &pc = ch.tables[op.table_id];
    std::unique_lock<std::mutex> lk(ch.mu);
    const double w0 = now_s();
    while (pc.data_age < need) {
      if (!ch.cv.wait_for(lk, std::chrono::milliseconds(kWaitWarnMs), [&] { return pc.data_age >= need; }) &&
          ch.id == 0)
        std::cerr << "machine " << process_id_ << " wait time out! Need: " << need << " Data age: " << pc.data_age
                  << std::endl;
    }
    waited += now_s() - w0;
    const gp_double_index *idx = op.host_index.data() + op.ch_start[ch.id];
    const size_t n = op.ch_size[ch.id];
    if (ch.id + 1 < channels_.size()) {
      if (n)
        GP_CALL(gp_host_gather_rows(cpu_buffer_.data(), pc.cpu.data->data(), idx, n, gp_double_index{0, 0},
                                    ROW_DATA_SIZE, op.num_vals_limit));
      continue;
    }
    const size_t vals = std::min(op.num_vals_limit, op.rows.size() * ROW_DATA_SIZE);
    for (size_t r0 = 0; r0 * ROW_DATA_SIZE < vals; r0 += kHostPieceRows) {
      const auto e = entries_in(idx, n, r0, r0 + kHostPieceRows);
      if (e.second > e.first)
        GP_CALL(gp_host_gather_rows(cpu_buffer_.data(), pc.cpu.data->data(), idx + e.first, e.second - e.first,
                                    gp_double_index{0, 0}, ROW_DATA_SIZE, op.num_vals_limit));
      const size_t f0 = r0 * ROW_DATA_SIZE, f1 = std::min(vals, (r0 + kHostPieceRows) * ROW_DATA_SIZE);
      GP_CALL(gp_memcpy_async(op.buffer.data() + f0, cpu_buffer_.data() + f0, (f1 - f0) * sizeof(float),
                              channels_[0]->stream->get()));
    }
  }
  channels_[0]->stream->sync();
  std::lock_guard<std::mutex> lk(stats_mu_);
  stats_.nr_read++;
  stats_.nr_read_host++;
  stats_.rows_read += op.rows.size();
  stats_.read_wait_time += waited;
  stats_.read_time += now_s() - t0;
}

// A host-tier op's Update: the app's rows (written by its device work on the
// null stream) come to the pinned host buffer, num_vals_limit floats
// (update_batch_param_cache, clientlib-data.cpp:309-323); then per channel,
// under its lock, the clock's host oplog (zeroed when created) += the op's
// rows through the host DoubleIndex, and with read-my-writes the host cache
// too (update_batch_cpu, :398-434).  The rows come down piece by piece, and
// each piece is added as soon as it has landed (a row's adds keep their op
// order: the pieces go in op-row order).
void ClientLib::update_batch_host(OpInfo &pre, iter_t clock) {
  const size_t vals = std::min(pre.num_vals_limit, pre.rows.size() * ROW_DATA_SIZE);
  Channel &ch0 = *channels_[0];
  ch0.app_written.record_default();
  GP_CALL(gp_stream_wait_event(ch0.stream->get(), ch0.app_written.get()));
  const size_t piece_vals = kHostPieceRows * ROW_DATA_SIZE;
  const size_t pieces = (vals + piece_vals - 1) / piece_vals;
  while (host_events_.size() < pieces) host_events_.push_back(std::make_unique<Event>());
  for (size_t k = 0; k < pieces; ++k) {
    const size_t f0 = k * piece_vals, f1 = std::min(vals, f0 + piece_vals);
    GP_CALL(gp_memcpy_async(cpu_buffer_.data() + f0, pre.buffer.data() + f0, (f1 - f0) * sizeof(float),
                            ch0.stream->get()));
    host_events_[k]->record(*ch0.stream);
  }
  // the clock's host oplogs (zeroed when new) while the rows come down
  std::vector<std::shared_ptr<HostBuf>> oplogs(channels_.size());
  for (auto &chp : channels_) {
    std::lock_guard<std::mutex> lk(chp->mu);
    HostTier &cpu = chp->tables[pre.table_id].cpu;
    if (cpu.num_rows) oplogs[chp->id] = get_host_oplog(cpu, clock);
  }
  for (size_t k = 0; k < pieces; ++k) {
    host_events_[k]->sync();
    for (auto &chp : channels_) {
      Channel &ch = *chp;
      const size_t n = pre.ch_size[ch.id];
      if (!n || !oplogs[ch.id]) continue;
      const gp_double_index *idx = pre.host_index.data() + pre.ch_start[ch.id];
      const auto e = entries_in(idx, n, k * kHostPieceRows, (k + 1) * kHostPieceRows);
      if (e.second == e.first) continue;
      std::lock_guard<std::mutex> lk(ch.mu);
      GP_CALL(gp_host_scatter_add_rows(oplogs[ch.id]->data(), cpu_buffer_.data(), idx + e.first,
                                       e.second - e.first, gp_double_index{0, 0}, ROW_DATA_SIZE,
                                       pre.num_vals_limit));
      if (config_.read_my_writes)
        GP_CALL(gp_host_scatter_add_rows(ch.tables[pre.table_id].cpu.data->data(), cpu_buffer_.data(),
                                         idx + e.first, e.second - e.first, gp_double_index{0, 0}, ROW_DATA_SIZE,
                                         pre.num_vals_limit));
    }
  }
}

// create_oplog_entry + zerofy_data_cpu (clientlib-data.cpp:412-417): a pooled
// host buffer once nothing (a pending push, the in-process server's bucket)
// references it.
std::shared_ptr<HostBuf> ClientLib::get_host_oplog(HostTier &cpu, iter_t clock) {
  auto it = cpu.oplog.find(clock);
  if (it != cpu.oplog.end()) return it->second;
  std::shared_ptr<HostBuf> buf;
  for (auto &b : cpu.oplog_pool)
    if (b.use_count() == 1) {
      buf = b;
      break;
    }
  if (!buf) {
    bool share = host_share_;
    if (share && ipc_fault_ == 2 && !ipc_fault_used_[2].exchange(true)) {
      std::cerr << "libgeeps: GEEPS_TEST_IPC_FAULT=refuse: shared host oplog refused\n";
      share = false;
    }
    cpu.oplog_pool.push_back(
        std::make_shared<HostBuf>(cpu.num_rows * ROW_DATA_SIZE, config_.pinned_cpu_memory != 0, share));
    buf = cpu.oplog_pool.back();
    if (host_share_ && !buf->shared()) {
      std::lock_guard<std::mutex> lk(stats_mu_);
      stats_.nr_host_share_refused++;
    }
  }
  buf->zero();
  cpu.oplog[clock] = buf;
  return buf;
}

void ClientLib::postread_batch(int handle) {
  check_handle(handle);
  OpInfo &op = opseq_[handle];
  GP_CHECK(op.type == OpInfo::POST_READ);
  OpInfo &pre = opseq_[op.prestep_handle];
  GP_CHECK(pre.type == OpInfo::READ);
  // GPU-resident local data is used in place, so `keep` needs no copy back
  // (the reference copies back only for CPU-placed local data).
  pre.in_use = false;
  if (pre.pin_server < 0) return;
  // A direct Read's pin ends: a version a refresh replaced meanwhile goes back
  // to its server once no direct Read pins it (outside ch.mu, as the reader
  // threads give versions back).  The app's device work that reads the buffer
  // was queued before this call, typically on the null stream, and may still
  // run: the event recorded here orders every later release of the version
  // after it (the mirror of Update's app_written).
  Channel &ch = *channels_[pre.direct_channel];
  const uint32_t s = (uint32_t)pre.pin_server;
  const int v = pre.pin_version;
  pre.pin_server = pre.pin_version = -1;
  if (!pre.read_done) pre.read_done = std::make_unique<Event>();
  pre.read_done->record_default();
  bool back = false;
  std::set<Event *> wait;
  {
    std::lock_guard<std::mutex> lk(ch.mu);
    ParamCache &pc = ch.tables[pre.table_id];
    auto it = pc.pins[s].find(v);
    GP_CHECK(it != pc.pins[s].end() && it->second > 0);
    pc.read_events[s][v].insert(pre.read_done.get());
    if (--it->second == 0) {
      pc.pins[s].erase(it);
      back = pc.deferred[s].erase(v) > 0;
      if (back) {
        wait.swap(pc.read_events[s][v]);
        pc.read_events[s].erase(v);
      }
    }
  }
  if (!back) return;
  for (Event *e : wait) e->sync();
  give_back(ch, s, pre.table_id, v);
  std::lock_guard<std::mutex> lk(stats_mu_);
  stats_.nr_read_pin_deferred++;
}

// ---------------------------------------------------------------------------
// PreUpdate / Update (clientlib.cpp:475-614; clientlib-data.cpp:304-396)
// ---------------------------------------------------------------------------
void ClientLib::preupdate_batch(RowOpVal **buffer, int handle) {
  check_handle(handle);
  OpInfo &op = opseq_[handle];
  GP_CHECK(op.type == OpInfo::PRE_WRITE);
  GP_CHECK(!op.local);
  GP_CHECK_MSG(!op.in_use, "PreUpdate of handle " << handle << " before its Update");
  op.in_use = true;
  op.direct_now = started_ && op.direct;
  if (op.direct_now) {
    // the clock's oplog slice of this op's rows (not zeroed: every row of it
    // is written by exactly one update op of the clock)
    Channel &ch = *channels_[op.direct_channel];
    std::lock_guard<std::mutex> lk(ch.mu);
    ParamCache &pc = ch.tables[op.table_id];
    auto oplog = get_oplog(pc, iteration_, ch.stream->get(), /*zero=*/false);
    ch.stream->sync();  // a fresh pool buffer's zero fill lands before the app writes
    *buffer = reinterpret_cast<RowOpVal *>(oplog->data() + op.direct_lo * ROW_DATA_SIZE);
    return;
  }
  *buffer = reinterpret_cast<RowOpVal *>(op.buffer.data());
}

std::shared_ptr<DeviceArray<float>> ClientLib::get_oplog(ParamCache &pc, iter_t clock,
                                                         gp_stream s, bool zero) {
  auto it = pc.oplog.find(clock);
  if (it != pc.oplog.end()) return it->second;
  // create_oplog_entry + zerofy_data_gpu (clientlib.cpp:265-280,
  // clientlib-data.cpp:356-371).  A pooled buffer is reused once nothing (the
  // in-process server's pending bucket included) references it.
  std::shared_ptr<DeviceArray<float>> buf;
  for (size_t k = 0; k < pc.oplog_pool.size(); ++k) {
    auto &b = pc.oplog_pool[k];
    if (b.use_count() != 1) continue;
    if (k < pc.oplog_bad.size() && pc.oplog_bad[k]) {
      // its export was refused or a server could not map it: a fresh buffer
      // takes its place (the old one is kept until Shutdown, since another
      // server may still have it mapped), exported anew to every server
      pc.retired.push_back(b);
      b = std::make_shared<DeviceArray<float>>(pc.num_rows * ROW_DATA_SIZE, kShared);
      pc.oplog_bad[k] = 0;
      if (k < pc.exported.size()) std::fill(pc.exported[k].begin(), pc.exported[k].end(), 0);
      zero = true;
    }
    buf = b;
    break;
  }
  if (!buf) {
    // (a same-node server maps it over IPC: a whole allocation)
    pc.oplog_pool.push_back(std::make_shared<DeviceArray<float>>(pc.num_rows * ROW_DATA_SIZE, kShared));
    buf = pc.oplog_pool.back();
    // a new buffer never shows uninitialised HBM: a direct-oplog PreUpdate
    // hands it to the app, and rows an app leaves unwritten then push zeros
    zero = true;
  }
  if (zero) GP_CALL(gp_zero(buf->data(), pc.num_rows * ROW_DATA_SIZE, s));
  pc.oplog[clock] = buf;
  return buf;
}

void ClientLib::update_batch(int handle) {
  check_handle(handle);
  OpInfo &op = opseq_[handle];
  GP_CHECK(op.type == OpInfo::WRITE);
  OpInfo &pre = opseq_[op.prestep_handle];
  GP_CHECK(pre.type == OpInfo::PRE_WRITE && !pre.local);
  GP_CHECK_MSG(pre.in_use, "Update of handle " << handle << " without PreUpdate");
  const double t0 = now_s();
  const iter_t clock = iteration_;
  if (pre.cpu) update_batch_host(pre, clock);
  for (auto &chp : channels_) {
    if (pre.cpu) break;
    Channel &ch = *chp;
    const size_t n = pre.ch_size[ch.id];
    std::lock_guard<std::mutex> lk(ch.mu);
    ParamCache &pc = ch.tables[pre.table_id];
    if (pc.num_rows == 0) continue;
    const bool fused = started_ && ch.init_ok[pre.table_id];
    // the app wrote its rows with its own device work, typically on the null
    // stream (the reference's worker ran on a blocking stream, which waited
    // for it implicitly): everything this Update queues, and the push and the
    // server's sum after it, comes after those writes
    if (n) {
      ch.app_written.record_default();
      GP_CALL(gp_stream_wait_event(ch.stream->get(), ch.app_written.get()));
    }
    auto oplog = get_oplog(pc, clock, ch.stream->get(), /*zero=*/!fused);
    // the rows the app wrote: its op buffer, or (direct) the oplog slice itself
    const bool in_place = pre.direct_now && (int)ch.id == pre.direct_channel;
    const float *x = in_place ? oplog->data() + pre.direct_lo * ROW_DATA_SIZE : pre.buffer.data();
    if (n) {
      // add_rows_from_double_index_gpu (clientlib-data.cpp:385-394) through the
      // op's row plan for this channel (its index, offset 0, num_vals_limit)
      const gp_row_plan plan = pre.plans[ch.id]->get();
      if (!in_place) {  // (in place: the app wrote these rows into the oplog itself)
        if (fused)
          GP_CALL(gp_scatter_init_rows_planned(oplog->data(), x, plan, ch.stream->get()));
        else
          GP_CALL(gp_scatter_add_rows_planned(oplog->data(), x, plan, ch.stream->get()));
      }
      if (config_.read_my_writes && pc.segmented) {
        // (unreachable today: read-my-writes refreshes are private copies, so
        // its cache is never segmented; the unplanned add has no repeat layers)
        GP_CHECK_MSG(!pre.repeats, "read-my-writes update of an op listing a row twice into a "
                                   "segmented cache");
        GP_CALL(gp_scatter_add_rows_segmented(&pc.segs, x,
                                              pre.index.data() + pre.ch_start[ch.id], n,
                                              gp_double_index{0, 0}, ROW_DATA_SIZE,
                                              pre.num_vals_limit, ch.stream->get()));
      } else if (config_.read_my_writes)
        GP_CALL(gp_scatter_add_rows_planned(pc.data.data(), x, plan, ch.stream->get()));
    }
    ch.stream->sync();
  }
  pre.in_use = false;
  const bool was_direct = pre.direct_now;
  pre.direct_now = false;
  {
    std::lock_guard<std::mutex> lk(stats_mu_);
    stats_.nr_update++;
    if (was_direct) stats_.nr_update_direct++;
    if (pre.cpu) stats_.nr_update_host++;
    stats_.rows_updated += pre.rows.size();
    stats_.update_time += now_s() - t0;
  }
  // After StartIterations the table is clocked at its last write
  // (reclaim_worker_update, clientlib-bg-access.cpp:534-538).
  if (started_ && op.table_last_write) clock_table(clock + 1, op.table_id);
}

// ---------------------------------------------------------------------------
// Clock (clientlib.cpp:282-314, 617-625) and the push (clientlib-data.cpp:436-522)
// ---------------------------------------------------------------------------
void ClientLib::iterate() {
  iteration_++;
  {
    std::lock_guard<std::mutex> lk(stats_mu_);
    stats_.nr_clock++;
  }
  if (started_) {
    // Every declared op of the iteration must have run (the reference's
    // background workers replay the whole sequence; a skipped op would stall
    // them), which is also what makes the fused oplog init safe.
    GP_CHECK_MSG(clock_handle_ < 0 || last_handle_ == clock_handle_ - 1,
                 "Clock() after handle " << last_handle_ << " but the iteration declares ops up to "
                                         << clock_handle_ - 1);
    last_handle_ = -1;
  } else {
    clock_all(iteration_);
  }
}

void ClientLib::clock_all(iter_t clock) {
  for (uint32_t t = 0; t < config_.num_tables; ++t) clock_table(clock, t);
}

void ClientLib::clock_table(iter_t clock, uint32_t table_id) {
  fast_clock_ = clock;
  const iter_t signalled = clock - 1;  // "clock c" means clock c-1 is finished
  for (auto &chp : channels_) push_updates(*chp, signalled, table_id);
}

void ClientLib::push_updates(Channel &ch, iter_t clock, uint32_t table_id) {
  const double t0 = now_s();
  std::shared_ptr<DeviceArray<float>> oplog;
  std::vector<size_t> starts, counts;
  std::shared_ptr<const std::vector<RowKey>> keys;  // immutable after FinishVirtualIteration
  size_t pool_id = 0;
  std::vector<uint8_t> *exported = nullptr;  // app thread only
  std::vector<uint8_t> *keys_sent = nullptr;  // app thread only
  std::vector<uint8_t> *bad = nullptr;        // app thread only
  // the host tier (empty unless gpu_memory_capacity placed rows there): its
  // oplog, server partition and the per-server frame keys [host | HBM]
  std::shared_ptr<HostBuf> hoplog;
  std::vector<size_t> cstarts, ccounts;
  std::vector<std::shared_ptr<std::vector<RowKey>>> frame_keys;
  bool tiers = false, zero_filled = false;
  // ... and, when the host oplog is shared memory, which same-node servers map
  // it (app thread only) and which of them could not (their NACKs)
  size_t hpool_id = 0;
  std::vector<uint8_t> *hexported = nullptr;
  std::vector<uint8_t> share_off;
  {
    std::lock_guard<std::mutex> lk(ch.mu);
    ParamCache &pc = ch.tables[table_id];
    HostTier &cpu = pc.cpu;
    tiers = cpu.num_rows > 0;
    if (tiers) {
      auto hit = cpu.oplog.find(clock);
      if (hit != cpu.oplog.end()) hoplog = hit->second;
      const bool any = hoplog || pc.oplog.count(clock);
      // a clock's push carries both tiers' rows (the server sums each shard
      // positionally): a tier no op updated this clock sends zeros
      if (any && !hoplog) hoplog = get_host_oplog(cpu, clock);
      if (any && !pc.oplog.count(clock) && pc.num_rows) {
        get_oplog(pc, clock, ch.stream->get(), /*zero=*/true);
        zero_filled = true;
      }
      cstarts = cpu.server_row_start;
      ccounts = cpu.server_num_rows;
      frame_keys = pc.frame_keys;
      if (hoplog && hoplog->shared()) {
        for (size_t k = 0; k < cpu.oplog_pool.size(); ++k)
          if (cpu.oplog_pool[k] == hoplog) hpool_id = k;
        if (cpu.exported.size() < cpu.oplog_pool.size())
          cpu.exported.resize(cpu.oplog_pool.size(), std::vector<uint8_t>(num_processes_, 0));
        hexported = &cpu.exported[hpool_id];
        share_off = ch.host_share_off;
      }
      // (the frames keep it alive; a same-node server's NACK needs it until
      // its refresh covers the clock, as the HBM oplog: recv_row_batch reclaims)
      bool ipc_servers = false;
      for (uint32_t s = 0; s < num_processes_; ++s) ipc_servers |= ipc_to(s);
      if (hoplog && !config_.read_my_writes && !ipc_servers) cpu.oplog.erase(clock);
    }
    if (pc.oplog_bad.size() < pc.oplog_pool.size()) pc.oplog_bad.resize(pc.oplog_pool.size(), 0);
    if (pc.exported.size() < pc.oplog_pool.size())
      pc.exported.resize(pc.oplog_pool.size(), std::vector<uint8_t>(num_processes_, 0));
    // servers that could not map a buffer (their NACK's resend went already):
    // it is replaced before its next use, and exported anew
    for (auto &nk : pc.ipc_nacked)
      if (nk.first < pc.oplog_pool.size()) {
        pc.exported[nk.first][nk.second] = 0;
        pc.oplog_bad[nk.first] = 1;
      }
    pc.ipc_nacked.clear();
    bad = &pc.oplog_bad;
    auto it = pc.oplog.find(clock);
    if (it != pc.oplog.end()) oplog = it->second;
    starts = pc.server_row_start;
    counts = pc.server_num_rows;
    keys = pc.row_keys;
    if (pc.ipc_keys_sent.size() < num_processes_) pc.ipc_keys_sent.assign(num_processes_, 0);
    keys_sent = &pc.ipc_keys_sent;
    bool ipc_readers = false;  // a same-node server reads its slice from this oplog
    for (uint32_t s = 0; s < num_processes_; ++s) ipc_readers |= ipc_to(s) && (counts[s] > 0 || tiers);
    if (oplog) {
      for (size_t k = 0; k < pc.oplog_pool.size(); ++k)
        if (pc.oplog_pool[k] == oplog) pool_id = k;
      if (pc.exported.size() < pc.oplog_pool.size())
        pc.exported.resize(pc.oplog_pool.size(), std::vector<uint8_t>(num_processes_, 0));
      exported = &pc.exported[pool_id];
      // reclaim_oplog now, unless it must outlive the refresh (read-my-writes
      // re-apply; same-node servers copying out of it): then recv_row_batch
      // reclaims it once every server's data age covers the clock.
      if (!config_.read_my_writes && !ipc_readers) pc.oplog.erase(it);
    }
  }
  if (zero_filled) ch.stream->sync();  // (the in-process server reads it on its own stream)
  size_t remote_bytes = 0;
  uint8_t ch_export_handle[kIpcHandleBytes];  // the export made for server s, when first
  for (uint32_t s = 0; s < num_processes_; ++s) {
    if (tiers && hoplog) {
      // A table with host-tier rows: every frame is [host rows of s][HBM rows
      // of s] (push_updates_param_cache, clientlib-data.cpp:487-509).  The
      // in-process server gets the host part and the oplog slice in place; a
      // same-node server the HBM part over IPC and the host part through the
      // shared host oplog (or in the frame); any other server an ordinary
      // socket frame (the reference's own path).
      const size_t ca = cstarts[s], cn = ccounts[s], a = starts[s], n = counts[s];
      if (s == process_id_) {
        UpdateBatch b;
        b.client_id = process_id_;
        b.clock = clock;
        b.table_id = table_id;
        b.keys = frame_keys[s]->data();
        b.keys_owner = frame_keys[s];
        b.num_rows = cn + n;
        b.split = cn;
        b.host_head = hoplog->data() + ca * ROW_DATA_SIZE;
        b.head_keepalive = hoplog;
        if (n) {
          b.device_rows = oplog->data() + a * ROW_DATA_SIZE;
          b.keepalive = oplog;
        }
        ch.server->post_updates(std::move(b));
        continue;
      }
      const bool host_shared = ipc_to(s) && cn && hexported && !share_off[s];
      if (ipc_to(s) && (oplog ? [&] {
            if ((*exported)[s]) return true;
            IpcRowsRef probe{};
            if (ipc_export(probe.handle, oplog->data(), 0)) {
              std::memcpy(ch_export_handle, probe.handle, sizeof probe.handle);
              return true;
            }
            (*bad)[pool_id] = 1;
            std::lock_guard<std::mutex> lk(stats_mu_);
            stats_.nr_ipc_export_refused++;
            return false;
          }() : host_shared)) {
        // Same-node server: the HBM rows stay in this oplog, mapped over IPC
        // (none: every row of the table in the host tier); the host-tier rows
        // stay in the shared host oplog, mapped by the server too (a 5th
        // part), or travel in the frame
        cs_clock_with_updates_batch_msg_t h{};
        h.cmd = CLOCK_WITH_UPDATES_BATCH;
        h.client_id = process_id_;
        h.clock = clock;
        h.table_id = table_id;
        HostRowsRef href{};
        if (host_shared) {
          href.buffer_id = ((uint64_t)table_id << 32) | (uint64_t)hpool_id;
          href.offset = ca * kRowBytes;
          href.bytes = cn * kRowBytes;
          if (!(*hexported)[s]) {
            href.has_handle = 1;
            href.handle = hoplog->shared()->handle();
            if (ipc_fault_ == 1 && !ipc_fault_used_[2].exchange(true)) {
              href.handle.tag[15] ^= 0x5a;  // the server's tag check fails
              std::cerr << "libgeeps: GEEPS_TEST_IPC_FAULT=tag: corrupted the tag of a shared host oplog\n";
            }
            (*hexported)[s] = 1;
          }
        }
        IpcRowsRef ref{};
        if (oplog) {
          ref.buffer_id = ((uint64_t)table_id << 32) | (uint64_t)pool_id;
          ref.offset = a * kRowBytes;
          ref.bytes = n * kRowBytes;
          if (!(*exported)[s]) {
            std::memcpy(ref.handle, ch_export_handle, sizeof ref.handle);
            ref.has_handle = 1;
            (*exported)[s] = 1;
          }
        }
        const bool with_keys = !(*keys_sent)[s];
        const Part keys_part =
            with_keys ? Part{frame_keys[s]->data(), (cn + n) * sizeof(RowKey)} : Part{nullptr, 0};
        if (host_shared) {
          send_to_server(ch, s, {Part{&h, sizeof h}, keys_part, Part{nullptr, 0}, Part{&ref, sizeof ref},
                                 Part{&href, sizeof href}});
          std::lock_guard<std::mutex> lk(stats_mu_);
          stats_.nr_host_shared++;
        } else {
          send_to_server(ch, s, {Part{&h, sizeof h}, keys_part, Part{hoplog->data() + ca * ROW_DATA_SIZE, cn * kRowBytes},
                                 Part{&ref, sizeof ref}});
        }
        (*keys_sent)[s] = 1;
        continue;
      }
      const size_t floats = (cn + n) * ROW_DATA_SIZE;
      if (ch.send_buf.size() < floats) ch.send_buf.resize(floats);
      if (cn) std::memcpy(ch.send_buf.data(), hoplog->data() + ca * ROW_DATA_SIZE, cn * kRowBytes);
      if (n)
        GP_CALL(gp_memcpy_async(ch.send_buf.data() + cn * ROW_DATA_SIZE, oplog->data() + a * ROW_DATA_SIZE,
                                n * kRowBytes, ch.stream->get()));
      ch.stream->sync();
      cs_clock_with_updates_batch_msg_t h{};
      h.cmd = CLOCK_WITH_UPDATES_BATCH;
      h.client_id = process_id_;
      h.clock = clock;
      h.table_id = table_id;
      send_to_server(ch, s, {Part{&h, sizeof h}, Part{frame_keys[s]->data(), (cn + n) * sizeof(RowKey)},
                             Part{ch.send_buf.data(), floats * sizeof(float)}});
      remote_bytes += floats * sizeof(float);
      continue;
    }
    if (!oplog) {
      // clock_broadcast: a CLOCK with no updates (encoder-decoder.cpp:85-100).
      if (s == process_id_) {
        ch.server->post_clock(process_id_, clock, table_id);
      } else {
        cs_clock_msg_t h{};
        h.cmd = CLOCK;
        h.client_id = process_id_;
        h.clock = clock;
        h.table_id = table_id;
        send_to_server(ch, s, {Part{&h, sizeof h}});
      }
      continue;
    }
    const size_t a = starts[s], n = counts[s];
    if (s == process_id_) {
      UpdateBatch b;
      b.client_id = process_id_;
      b.clock = clock;
      b.table_id = table_id;
      b.keys = keys->data() + a;
      b.num_rows = n;
      b.keys_owner = keys;
      b.device_rows = oplog->data() + a * ROW_DATA_SIZE;
      b.keepalive = oplog;  // zero-copy: the server reads the oplog slice in place
      ch.server->post_updates(std::move(b));
    } else if (ipc_to(s) && [&] {
                 if ((*exported)[s]) return true;
                 IpcRowsRef probe{};
                 if (ipc_export(probe.handle, oplog->data(), 0)) {
                   std::memcpy(ch_export_handle, probe.handle, sizeof probe.handle);
                   return true;
                 }
                 // the runtime refused the export: this slice goes by socket,
                 // and a fresh buffer replaces this one on its next use
                 (*bad)[pool_id] = 1;
                 std::lock_guard<std::mutex> lk(stats_mu_);
                 stats_.nr_ipc_export_refused++;
                 return false;
               }()) {
      // Same-node server: it copies its slice straight out of this oplog.
      cs_clock_with_updates_batch_msg_t h{};
      h.cmd = CLOCK_WITH_UPDATES_BATCH;
      h.client_id = process_id_;
      h.clock = clock;
      h.table_id = table_id;
      IpcRowsRef ref{};
      // unique per client across tables: the server maps buffers by this id
      ref.buffer_id = ((uint64_t)table_id << 32) | (uint64_t)pool_id;
      ref.offset = a * kRowBytes;
      ref.bytes = n * kRowBytes;
      if (!(*exported)[s]) {
        std::memcpy(ref.handle, ch_export_handle, sizeof ref.handle);
        ref.has_handle = 1;
        (*exported)[s] = 1;
        if (ipc_log())
          std::cerr << "libgeeps ipc export oplog: client " << process_id_ << " ch " << ch.id << " server " << s
                    << " buffer " << ref.buffer_id << " at " << static_cast<void *>(oplog->data()) << " bytes "
                    << oplog->bytes() << "\n";
      }
      const bool with_keys = !(*keys_sent)[s];
      send_to_server(ch, s, {Part{&h, sizeof h},
                             with_keys ? Part{keys->data() + a, n * sizeof(RowKey)} : Part{nullptr, 0},
                             Part{nullptr, 0}, Part{&ref, sizeof ref}});
      (*keys_sent)[s] = 1;
    } else {
      const size_t floats = n * ROW_DATA_SIZE;
      if (ch.send_buf.size() < floats) ch.send_buf.resize(floats);
      if (floats)
        copy_out_in_pieces(ch.send_buf.data(), oplog->data() + a * ROW_DATA_SIZE, floats * 4, *ch.stream,
                           ch.send_events);
      cs_clock_with_updates_batch_msg_t h{};
      h.cmd = CLOCK_WITH_UPDATES_BATCH;
      h.client_id = process_id_;
      h.clock = clock;
      h.table_id = table_id;
      send_to_server_chunked(ch, s, {Part{&h, sizeof h}, Part{keys->data() + a, n * sizeof(RowKey)},
                                     Part{ch.send_buf.data(), floats * 4}},
                             ch.send_events);
      remote_bytes += floats * 4;
    }
  }
  std::lock_guard<std::mutex> lk(stats_mu_);
  stats_.nr_push++;
  stats_.bytes_pushed_remote += remote_bytes;
  stats_.push_time += now_s() - t0;
}

void ClientLib::reclaim_oplogs(ParamCache &pc, iter_t upto) {
  for (auto it = pc.oplog.begin(); it != pc.oplog.end() && it->first <= upto;)
    it = pc.oplog.erase(it);
  for (auto it = pc.cpu.oplog.begin(); it != pc.cpu.oplog.end() && it->first <= upto;)
    it = pc.cpu.oplog.erase(it);
}

// recv_row_batch + recv_row_batch_gpu + server_clock_cbk
// (clientlib-data.cpp:51-151, clientlib-cbk.cpp:81-104).
std::vector<int> ClientLib::recv_row_batch(uint32_t channel, uint32_t server_id,
                                           uint32_t table_id, iter_t data_age, iter_t self_clock,
                                           const float *rows, size_t num_rows, int version,
                                           DeviceArray<float> *landing, const float *host_rows) {
  const double t0 = now_s();
  Channel &ch = *channels_[channel];
  std::vector<int> released;
  std::set<Event *> read_waits;
  bool in_place = false, staged = false;
  {
    std::lock_guard<std::mutex> lk(ch.mu);
    GP_CHECK_LT(table_id, ch.tables.size());
    ParamCache &pc = ch.tables[table_id];
    GP_CHECK_LT(server_id, num_processes_);
    // An empty reply means the server has seen no updates for the table yet:
    // the shard is all zeros, as the freshly zeroed cache already is.  With a
    // host tier the shard is [its host-tier rows][its HBM-tier rows].
    HostTier &cpu = pc.cpu;
    const size_t split = cpu.num_rows ? cpu.server_num_rows[server_id] : 0;
    GP_CHECK_MSG(num_rows == split + pc.server_num_rows[server_id] || num_rows == 0,
                 "refresh of " << num_rows << " rows, expected " << split + pc.server_num_rows[server_id]);
    iter_t &age = pc.per_server_data_age[server_id];
    GP_CHECK_MSG(data_age > age, "old or duplicate data received: " << data_age << " vs " << age);
    GP_CHECK_LE(data_age, self_clock);
    age = data_age;
    // server_clock_cbk: oplogs the servers have all applied can go.
    GP_CHECK_LE(pc.server_clock[server_id], data_age);
    pc.server_clock[server_id] = data_age;
    const iter_t min_clock = *std::min_element(pc.server_clock.begin(), pc.server_clock.end());
    if (min_clock > pc.server_clock_min) {
      reclaim_oplogs(pc, min_clock);
      pc.server_clock_min = min_clock;
    }
    if (num_rows && split) {
      // recv_row_batch_cpu (clientlib-data.cpp:153-189): the host-tier part
      // into the host cache -- from the socket frame's host copy, or device to
      // host from the master version -- then with read-my-writes this
      // client's own unreflected host oplogs on top, clock by clock.
      float *dst = cpu.data->data() + cpu.server_row_start[server_id] * ROW_DATA_SIZE;
      if (host_rows) {
        std::memcpy(dst, host_rows, split * kRowBytes);
      } else {
        GP_CALL(gp_memcpy_async(dst, rows, split * kRowBytes, ch.svc_stream->get()));
        ch.svc_stream->sync();
      }
      if (config_.read_my_writes)
        for (iter_t c = self_clock + 1, fc = fast_clock_.load(); c <= fc; ++c) {
          auto it = cpu.oplog.find(c);
          if (it != cpu.oplog.end())
            GP_CALL(gp_host_add(split * ROW_DATA_SIZE, dst,
                                it->second->data() + cpu.server_row_start[server_id] * ROW_DATA_SIZE));
        }
      // the rest is the HBM tier's part of the shard
      rows += split * ROW_DATA_SIZE;
      if (host_rows) host_rows += split * ROW_DATA_SIZE;
      num_rows -= split;
      if (num_rows == 0 && version >= 0) released.push_back(version);  // nothing of it read in place
    }
    bool own_buf = !pc.shard_buf.empty() && pc.shard_buf[server_id].data();
    if (num_rows && !own_buf && pc.data.size() == 0 && !(version >= 0 && !config_.read_my_writes &&
                                                          !ch.stage_refresh_from[server_id])) {
      // a copied refresh from a server whose shard this cache reads in place
      // (its export of the version was refused, IPC recovery): the shard
      // gets a buffer of its own
      if (pc.shard_buf.empty()) pc.shard_buf.resize(num_processes_);
      pc.shard_buf[server_id].resize(num_rows * ROW_DATA_SIZE);
      own_buf = true;
      rebuild_segments(pc);
    }
    if (num_rows == 0 && pc.num_rows && pc.data.size() == 0 && !own_buf) {
      // An empty shard reads as zeros from the cache's own rows, which a
      // cache that takes every refresh in place has not allocated yet.
      pc.data.resize(pc.num_rows * ROW_DATA_SIZE);
      GP_CALL(gp_zero(pc.data.data(), pc.data.size(), ch.svc_stream->get()));
      ch.svc_stream->sync();
      rebuild_segments(pc);
    }
    // a replaced version goes back now, or at the PostRead of the last direct
    // Read pinning it; either way after the app's device work on the direct
    // Reads' buffers (their PostRead events, waited on below)
    auto retire = [&](int v) {
      if (pc.pins[server_id].count(v)) {
        pc.deferred[server_id].insert(v);
        return;
      }
      auto ev = pc.read_events[server_id].find(v);
      if (ev != pc.read_events[server_id].end()) {
        read_waits.insert(ev->second.begin(), ev->second.end());
        pc.read_events[server_id].erase(ev);
      }
      released.push_back(v);
    };
    if (num_rows) {
      const int prev = pc.live_ver[server_id];
      staged = version >= 0 && ch.stage_refresh_from[server_id];
      if (version >= 0 && !config_.read_my_writes && !staged) {
        // The server's published master version becomes the live copy of
        // this shard, read in place by the segmented gather: no copy.  It is
        // never rewritten while we hold it; the one it replaces goes back.
        in_place = true;
        if (prev != version) {
          if (prev >= 0) retire(prev);
          pc.live_ver[server_id] = version;
          pc.live_ptr[server_id] = rows;
          rebuild_segments(pc);
        }
      } else {
        // Copy into the cache (recv_row_batch_gpu, clientlib-data.cpp:110-151):
        // rows from a socket; a same-node server on another GPU (staged: one
        // peer copy over xGMI per refresh, then every Read of the clock
        // gathers from local HBM); or read-my-writes, which re-applies this
        // client's own not-yet-reflected updates on top of the shard and so
        // needs a private copy (clientlib-data.cpp:132-150: cublasSaxpy -> gp_add).
        const size_t floats = num_rows * ROW_DATA_SIZE;
        GP_CHECK_MSG(own_buf || pc.data.size() == pc.num_rows * ROW_DATA_SIZE,
                     "copied refresh from server " << server_id << " into an unallocated cache");
        float *dst = own_buf ? pc.shard_buf[server_id].data()
                             : pc.data.data() + pc.server_row_start[server_id] * ROW_DATA_SIZE;
        bool swapped = false;
        if (own_buf && landing && landing->data() == rows && landing->size() >= floats) {
          // the reader's landing buffer holds the refreshed shard: it becomes
          // the shard's buffer and the old one the reader's next landing
          // buffer (every Read of the old one finished under this lock)
          pc.shard_buf[server_id].swap(*landing);
          swapped = true;
          rebuild_segments(pc);
        }
        std::vector<const float *> own;  // read-my-writes: the unreflected clocks' oplog slices, in order
        if (config_.read_my_writes)
          for (iter_t c = self_clock + 1, fc = fast_clock_.load(); c <= fc; ++c) {
            auto it = pc.oplog.find(c);
            if (it != pc.oplog.end()) own.push_back(it->second->data() + pc.server_row_start[server_id] * ROW_DATA_SIZE);
          }
        if (swapped) {
          // (no read-my-writes here: nothing to re-apply)
        } else if (!own.empty()) {
          // read-my-writes: copy and re-apply in one pass, dst = ((shard +
          // own[0]) + own[1]) + ..., the bits of a copy followed by one add per
          // oplog (clientlib-data.cpp:123-150), through the N-way sum kernels
          GP_CALL(gp_bucket_sum_into(dst, rows, own.data(), (int)own.size(), floats, ch.svc_stream->get()));
        } else {
          GP_CALL(gp_memcpy_async(dst, rows, num_rows * kRowBytes, ch.svc_stream->get()));
        }
        if (!swapped) ch.svc_stream->sync();
        if (version >= 0) released.push_back(version);  // copied: give it back now
        if (prev >= 0) {
          retire(prev);
          pc.live_ver[server_id] = -1;
          pc.live_ptr[server_id] = nullptr;
          rebuild_segments(pc);
        }
      }
    }
    pc.data_age = *std::min_element(pc.per_server_data_age.begin(), pc.per_server_data_age.end());
  }
  ch.cv.notify_all();
  for (Event *e : read_waits) e->sync();  // before the caller gives `released` back
  std::lock_guard<std::mutex> lk(stats_mu_);
  stats_.nr_refresh++;
  if (in_place) stats_.nr_refresh_in_place++;
  if (staged) stats_.nr_refresh_staged++;
  stats_.refresh_time += now_s() - t0;
  return released;
}

// The cache as row ranges: each server's shard is read from the cache's own
// `data` or in place from the server's live master version; neighbouring
// ranges of `data` merge.
void ClientLib::rebuild_segments(ParamCache &pc) {
  gp_row_segments t{};
  bool any_in_place = false;
  const float *next_flat = nullptr;  // where a merged `data` range would continue
  for (uint32_t s = 0; s < num_processes_; ++s) {
    const size_t n = pc.server_num_rows[s];
    if (n == 0) continue;
    const size_t first = pc.server_row_start[s];
    const bool in_place = !pc.live_ver.empty() && pc.live_ver[s] >= 0;
    // a shard of its own buffer (shard_buf) is a segment of its own too
    const bool own = !pc.shard_buf.empty() && pc.shard_buf[s].data();
    // (a shard neither in place nor copied yet is never read: see Read's wait)
    const float *base = in_place ? pc.live_ptr[s]
                        : own    ? pc.shard_buf[s].data()
                        : pc.data.data() ? pc.data.data() + first * ROW_DATA_SIZE : nullptr;
    any_in_place = any_in_place || in_place || own;
    if (t.count && base == next_flat && !in_place && !own) {
      next_flat = base + n * ROW_DATA_SIZE;
      continue;
    }
    GP_CHECK_MSG(t.count < GP_MAX_SEGMENTS, "param cache split into more than "
                                                << GP_MAX_SEGMENTS << " segments");
    t.first_row[t.count] = t.count ? first : 0;
    t.base[t.count] = const_cast<float *>(base);
    ++t.count;
    next_flat = in_place || own || !base ? nullptr : base + n * ROW_DATA_SIZE;
  }
  pc.segs = t;
  pc.segmented = any_in_place;
}

// ---------------------------------------------------------------------------
// stats / shutdown (clientlib.cpp:185-263)
// ---------------------------------------------------------------------------
std::string ClientLib::json_stats() {
  std::ostringstream o;
  {
    std::lock_guard<std::mutex> lk(stats_mu_);
    o << "{\"process_id\": " << process_id_ << ", \"client\": " << stats_.to_json()
      << ", \"servers\": [";
  }
  for (size_t c = 0; c < channels_.size(); ++c)
    o << (c ? ", " : "") << channels_[c]->server->stats_json();
  o << "]}";
  const std::string json = o.str();
  if (!config_.output_dir.empty()) {
    std::ofstream f(config_.output_dir + "/json_stats." + std::to_string(process_id_),
                    std::ofstream::out | std::ofstream::app);
    f << json << std::endl;
  }
  return json;
}

// Shutdown handshake: every client tells every server it is done; a server
// acknowledges all clients once all have; each client's reader, having handled
// that acknowledgement (and every frame before it), answers with
// kCmdReaderDone; each process tears down once its readers of both kinds are
// done.  A peer therefore never sees a connection close while it still expects
// a message, and no process frees a buffer whose IPC handle a peer has yet to
// open.
void ClientLib::shutdown() {
  if (stopping_.exchange(true)) return;
  for (auto &chp : channels_) {
    Channel &ch = *chp;
    for (uint32_t s = 0; s < num_processes_; ++s) {
      if (s == process_id_) {
        ch.server->post_shutdown(process_id_);
      } else {
        cs_clock_msg_t h{};
        h.cmd = SHUTDOWN;
        h.client_id = process_id_;
        send_to_server(ch, s, {Part{&h, sizeof h}});
      }
    }
  }
  for (auto &chp : channels_) chp->server->wait_shutdown();
  for (auto &chp : channels_) {
    for (auto &t : chp->client_readers)
      if (t.joinable()) t.join();
    for (auto &t : chp->server_readers)
      if (t.joinable()) t.join();
    chp->server->stop();
    for (auto &m : chp->ipc_oplogs)
      for (auto &kv : m) gp_ipc_close_handle(kv.second);
    for (auto &pc : chp->tables)
      for (auto &per_server : pc.server_versions)
        for (auto &kv : per_server) gp_ipc_close_handle(kv.second);
    for (int fd : chp->server_fd) close_fd(fd);
    for (int fd : chp->client_fd) close_fd(fd);
    close_fd(chp->listen_fd);
  }
  GP_CALL(gp_device_synchronize());
}

void ClientLib::quiesce() {
  if (stopping_.load()) return;
  for (auto &chp : channels_) chp->server->drain();
  gp_device_synchronize();
}

}  // namespace geeps
