// ClientLib — see client.hpp: construction, the per-clock API (iterate /
// clock), stats and Shutdown.  Reference: src/client/clientlib.cpp.
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

ClientLib *client_lib = nullptr;

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
    << ", \"nr_update_host_init\": " << nr_update_host_init << ", \"nr_read_host_run\": " << nr_read_host_run
    << ", \"nr_update_host_run\": " << nr_update_host_run
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
  const char *runs = std::getenv("GEEPS_HOST_RUNS");
  host_runs_ = !(runs && std::string(runs) == "0");
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
    ch->ipc_parked.resize(num_processes_);
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
    for (auto &parked : chp->ipc_parked)
      for (void *p : parked) gp_ipc_close_handle(p);
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
