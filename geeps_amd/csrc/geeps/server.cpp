// Tablet server — see server.hpp.  Reference: src/server/tablet-server.cpp.
#include "server.hpp"

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <future>
#include <iostream>
#include <sstream>

#include "check.hpp"

namespace geeps {

namespace {
double now_s() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

// How long free_version waits with no release at all before it gives up:
// GEEPS_VERSION_WAIT_S seconds, default 1800 (a paused worker -- a
// checkpoint, a long evaluation -- must not kill the job, ADVICE r03, but a
// dead or stuck reader must not hang it forever either: it fails with the
// holders matrix); 0 = no limit, the 12-s warnings only.  Every
// release restarts the clock.  The tests set 60 s.
double version_wait_limit_s() {
  static const double limit = [] {
    const char *v = std::getenv("GEEPS_VERSION_WAIT_S");
    const double d = v ? std::atof(v) : 1800.0;
    return d > 0 ? d : 0.0;
  }();
  return limit;
}
}  // namespace

std::string ServerStats::to_json() const {
  std::ostringstream o;
  o << "{\"nr_update\": " << nr_update << ", \"nr_local_update\": " << nr_local_update
    << ", \"nr_clock\": " << nr_clock << ", \"nr_refresh\": " << nr_refresh
    << ", \"nr_apply_launches\": " << nr_apply_launches
    << ", \"nr_apply_out_of_place\": " << nr_apply_out_of_place
    << ", \"nr_buckets_applied\": " << nr_buckets_applied
    << ", \"nr_versions\": " << nr_versions
    << ", \"nr_peer_staged\": " << nr_peer_staged
    << ", \"version_wait_time\": " << version_wait_time
    << ", \"apply_time\": " << apply_time << ", \"stage_time\": " << stage_time
    << ", \"refresh_time\": " << refresh_time << "}";
  return o.str();
}

TabletServer::TabletServer(uint32_t server_id, uint32_t channel_id, uint32_t num_clients,
                           uint32_t num_tables, ClientSink *sink, int device,
                           gp_stream stream)
    : server_id_(server_id),
      channel_id_(channel_id),
      num_clients_(num_clients),
      sink_(sink),
      device_(device),
      stream_(stream) {
  GP_CHECK(sink_);
  GP_CHECK(num_clients_ > 0);
  tables_.resize(num_tables);
  for (auto &t : tables_) t.vec_clock.assign(num_clients_, INITIAL_DATA_AGE);
  copy_streams_.resize(num_clients_);
  thread_ = std::thread([this] { run(); });
}

TabletServer::~TabletServer() { stop(); }

void TabletServer::post_updates(UpdateBatch &&batch) {
  Msg m{Msg::kUpdates, std::move(batch)};
  {
    std::lock_guard<std::mutex> lk(mu_);
    queue_.push_back(std::move(m));
  }
  cv_.notify_one();
}

void TabletServer::post_clock(uint32_t client_id, iter_t clock, uint32_t table_id) {
  Msg m{Msg::kClock, UpdateBatch{}};
  m.client_id = client_id;
  m.clock = clock;
  m.table_id = table_id;
  {
    std::lock_guard<std::mutex> lk(mu_);
    queue_.push_back(std::move(m));
  }
  cv_.notify_one();
}

void TabletServer::post_shutdown(uint32_t client_id) {
  Msg m{Msg::kShutdown, UpdateBatch{}};
  m.client_id = client_id;
  {
    std::lock_guard<std::mutex> lk(mu_);
    queue_.push_back(std::move(m));
  }
  cv_.notify_one();
}

void TabletServer::release(uint32_t client_id, uint32_t table_id, int version) {
  std::lock_guard<std::mutex> lk(hold_mu_);
  GP_CHECK_LT(table_id, tables_.size());
  GP_CHECK_LT(client_id, num_clients_);
  DataTable &t = tables_[table_id];
  GP_CHECK_MSG(version >= 0 && (size_t)version < t.holders.size() && t.holders[version][client_id],
               "client " << client_id << " releases master version " << version << " of table "
                         << table_id << " it does not hold");
  t.holders[version][client_id] = 0;
  ++releases_;
  release_cv_.notify_all();
}

void TabletServer::release_all(uint32_t client_id) {
  std::lock_guard<std::mutex> lk(hold_mu_);
  GP_CHECK_LT(client_id, num_clients_);
  for (auto &t : tables_)
    for (auto &h : t.holders) h[client_id] = 0;
  ++releases_;
  release_cv_.notify_all();
}

void TabletServer::held_version(uint32_t client_id, uint32_t table_id, int version, const float **rows,
                                size_t *num_rows, const RowKey **keys) {
  std::lock_guard<std::mutex> lk(hold_mu_);
  GP_CHECK_LT(table_id, tables_.size());
  GP_CHECK_LT(client_id, num_clients_);
  DataTable &t = tables_[table_id];
  GP_CHECK_MSG(version >= 0 && (size_t)version < t.holders.size() && t.holders[version][client_id],
               "client " << client_id << " asks for a resend of master version " << version << " of table "
                         << table_id << " it does not hold");
  *rows = t.versions[version]->data();
  *num_rows = t.row_count;
  *keys = t.row_keys.data();  // (immutable once the first update defined the shard)
}

void TabletServer::wait_shutdown() {
  std::unique_lock<std::mutex> lk(mu_);
  shutdown_cv_.wait(lk, [this] { return shutdown_done_; });
}

void TabletServer::drain() {
  if (!thread_.joinable()) return;
  std::promise<void> p;
  auto f = p.get_future();
  Msg m{Msg::kDrain, UpdateBatch{}};
  m.done = [&p] { p.set_value(); };
  {
    std::lock_guard<std::mutex> lk(mu_);
    queue_.push_back(std::move(m));
  }
  cv_.notify_one();
  f.wait();
}

std::string TabletServer::stats_json() {
  if (!thread_.joinable()) return stats_.to_json();
  std::promise<std::string> p;
  auto f = p.get_future();
  Msg m{Msg::kDrain, UpdateBatch{}};
  m.done = [this, &p] { p.set_value(stats_.to_json()); };
  {
    std::lock_guard<std::mutex> lk(mu_);
    queue_.push_back(std::move(m));
  }
  cv_.notify_one();
  return f.get();
}

void TabletServer::stop() {
  if (!thread_.joinable()) return;
  {
    std::lock_guard<std::mutex> lk(mu_);
    queue_.push_back(Msg{Msg::kStop, UpdateBatch{}});
  }
  cv_.notify_one();
  thread_.join();
}

void TabletServer::run() {
  GP_CALL(gp_set_device(device_));
  for (;;) {
    Msg m{Msg::kStop, UpdateBatch{}};
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [this] { return !queue_.empty(); });
      m = std::move(queue_.front());
      queue_.pop_front();
    }
    switch (m.kind) {
      case Msg::kUpdates: {
        // CLOCK_WITH_UPDATES_BATCH: update_row_batch() then clock()
        // (server-encoder-decoder.cpp:104-110).
        const uint32_t c = m.batch.client_id, tb = m.batch.table_id;
        const iter_t ck = m.batch.clock;
        update_row_batch(m.batch);
        clock(c, ck, tb);
        break;
      }
      case Msg::kClock:
        clock(m.client_id, m.clock, m.table_id);
        break;
      case Msg::kShutdown:
        // Per-connection order guarantees the client's updates and clocks
        // were all processed before its SHUTDOWN.
        if (++shutdown_count_ == num_clients_) {
          for (auto &t : tables_) apply_pending(t);
          for (uint32_t c = 0; c < num_clients_; ++c) sink_->shutdown_ack(c);
          std::lock_guard<std::mutex> lk(mu_);
          shutdown_done_ = true;
          shutdown_cv_.notify_all();
        }
        break;
      case Msg::kDrain:
        if (m.done) m.done();
        break;
      case Msg::kStop:
        return;
    }
  }
}

// A staging bucket no pending bucket references.  At most kMaxPendingBuckets
// exist per table (the queue is applied when it reaches that many, which
// frees them all); the client's memory plan counts them (client_viter.cpp,
// FinishVirtualIteration).
std::shared_ptr<DeviceArray<float>> TabletServer::stage_buffer(DataTable &t) {
  for (auto &b : t.stage_pool)
    if (b.use_count() == 1) return b;  // not referenced by a pending bucket
  GP_CHECK_LT(t.stage_pool.size(), kMaxPendingBuckets);
  t.stage_pool.push_back(std::make_shared<DeviceArray<float>>(t.row_count * ROW_DATA_SIZE));
  return t.stage_pool.back();
}

// TabletStorage::update_row_batch (src/server/tablet-server.cpp:81-117).
void TabletServer::update_row_batch(UpdateBatch &b) {
  const size_t batch_size = b.num_rows;
  stats_.nr_update += batch_size;
  if (b.client_id == server_id_) stats_.nr_local_update += batch_size;
  GP_CHECK_LT(b.table_id, tables_.size());
  DataTable &t = tables_[b.table_id];
  GP_CHECK_LT(b.client_id, t.vec_clock.size());
  const iter_t cur = t.vec_clock[b.client_id];
  GP_CHECK_MSG(cur == INITIAL_DATA_AGE || b.clock == cur + 1,
               "CS clocks out of sync, client = " << b.client_id << " clock = " << b.clock
                                                  << " cur_clock = " << cur);
  if (batch_size == 0) return;
  if (t.row_count == 0) {
    // The first message defines the shard: zeroed master, keys copied
    // (tablet-server.cpp:108-114).  Later messages are summed positionally.
    GP_CHECK_MSG(b.keys, "first update batch of table " << b.table_id << " from client "
                                                          << b.client_id << " carries no row keys");
    t.row_count = batch_size;
    t.cur = free_version(t);
    t.cur_published = false;
    GP_CALL(gp_zero(t.versions[t.cur]->data(), batch_size * ROW_DATA_SIZE, stream_));
    t.row_keys.assign(b.keys, b.keys + batch_size);
  }
  GP_CHECK_EQ(t.row_count, batch_size);

  Pending p;
  if (b.split) {
    // Host-tier rows first, then the HBM-tier slice (the in-process client of
    // a table with a host tier): both into one staging bucket, so the sum
    // reads one contiguous bucket as for any client.
    GP_CHECK_LE(b.split, batch_size);
    const double t0 = now_s();
    auto stage = stage_buffer(t);
    GP_CALL(gp_memcpy_async(stage->data(), b.host_head, b.split * ROW_DATA_SIZE * sizeof(float), stream_));
    if (batch_size > b.split) {
      GP_CHECK(b.device_rows);
      GP_CALL(gp_memcpy_async(stage->data() + b.split * ROW_DATA_SIZE, b.device_rows,
                              (batch_size - b.split) * ROW_DATA_SIZE * sizeof(float), stream_));
    }
    GP_CALL(gp_stream_synchronize(stream_));  // the host part is released when `b` dies
    stats_.stage_time += now_s() - t0;
    p.rows = stage->data();
    p.keepalive = stage;
  } else if (b.device_rows && b.stage) {
    // A same-node peer on another GPU: copy its slice into local HBM now (a
    // peer copy over xGMI on the copy stream, overlapped with whatever else
    // arrives), so the sum streams local HBM only.  apply_pending waits for it.
    auto stage = stage_buffer(t);
    GP_CHECK_LT(b.client_id, num_clients_);
    auto &cs = copy_streams_[b.client_id];
    if (!cs) cs = std::make_unique<Stream>();
    GP_CALL(gp_memcpy_async(stage->data(), b.device_rows, batch_size * ROW_DATA_SIZE * sizeof(float), cs->get()));
    p.staged = std::make_shared<Event>();
    p.staged->record(*cs);
    p.rows = stage->data();
    p.keepalive = stage;
    stats_.nr_peer_staged++;
  } else if (b.device_rows) {
    // In-process client: its oplog slice, read in place (keepalive holds it).
    // Same-node peer on this GPU: its oplog slice through the IPC mapping,
    // also read in place.
    p.rows = b.device_rows;
    p.keepalive = std::move(b.keepalive);
  } else {
    GP_CHECK(b.host_rows && b.host_rows->size() >= batch_size * ROW_DATA_SIZE);
    const double t0 = now_s();
    auto stage = stage_buffer(t);
    GP_CALL(gp_memcpy_async(stage->data(), b.host_rows->data(),
                            batch_size * ROW_DATA_SIZE * sizeof(float), stream_));
    GP_CALL(gp_stream_synchronize(stream_));  // host buffer is released when `b` dies
    stats_.stage_time += now_s() - t0;
    p.rows = stage->data();
    p.keepalive = stage;
  }
  t.pending.push_back(std::move(p));
  if (t.pending.size() >= kMaxPendingBuckets) apply_pending(t);
}

// A version no client holds, other than the current one; a new one when
// every version is held and fewer than clients + 2 exist; otherwise wait for
// a release (see server.hpp: it comes from a reader thread catching up, or
// from a direct Read's PostRead).  With GEEPS_VERSION_WAIT_S set the wait is
// bounded: every release restarts the clock, and after that long with none the
// server fails loudly with the holders matrix (a reader thread stuck or dead
// without a SHUTDOWN) instead of stalling the channel forever.
int TabletServer::free_version(DataTable &t) {
  std::unique_lock<std::mutex> lk(hold_mu_);
  const double t0 = now_s();
  double progress_t = t0;
  uint64_t seen = releases_;
  for (;;) {
    for (size_t v = 0; v < t.versions.size(); ++v) {
      if ((int)v == t.cur) continue;
      bool held = false;
      for (uint8_t h : t.holders[v]) held = held || h;
      if (!held) {
        stats_.version_wait_time += now_s() - t0;
        return (int)v;
      }
    }
    if (t.versions.size() < (size_t)num_clients_ + 2) {
      // (same-node clients map it over IPC: a whole allocation)
      t.versions.push_back(std::make_unique<DeviceArray<float>>(t.row_count * ROW_DATA_SIZE, kShared));
      t.holders.emplace_back(num_clients_, 0);
      stats_.nr_versions++;
      return (int)t.versions.size() - 1;
    }
    if (release_cv_.wait_for(lk, std::chrono::milliseconds(12000)) == std::cv_status::timeout)
      std::cerr << "tablet server " << server_id_ << " channel " << channel_id_
                << ": every master version is held; waiting for a client to release one\n";
    const double now = now_s();
    if (releases_ != seen) {
      seen = releases_;
      progress_t = now;
    } else if (version_wait_limit_s() > 0 && now - progress_t > version_wait_limit_s()) {
      std::ostringstream o;
      o << "tablet server " << server_id_ << " channel " << channel_id_ << ": no master version "
        << "released for " << (now - progress_t) << " s (GEEPS_VERSION_WAIT_S); holders "
        << "[version][client]:";
      for (size_t v = 0; v < t.holders.size(); ++v) {
        o << " v" << v << ((int)v == t.cur ? "*" : "") << "=";
        for (uint8_t h : t.holders[v]) o << (h ? '1' : '0');
      }
      GP_CHECK_MSG(false, o.str());
    }
  }
}

// All queued buckets in arrival order, one launch: master = ((m + b0) + b1) ...
// in place, or into a fresh version when clients may be reading the current
// one (same bits: gp_bucket_sum_into).
void TabletServer::apply_pending(DataTable &t) {
  if (t.pending.empty()) return;
  const double t0 = now_s();
  std::vector<const float *> ptrs;
  ptrs.reserve(t.pending.size());
  for (auto &p : t.pending) {
    ptrs.push_back(p.rows);
    if (p.staged) GP_CALL(gp_stream_wait_event(stream_, p.staged->get()));  // peer copy landed
  }
  const float *in = t.versions[t.cur]->data();
  if (t.cur_published) {
    bool held = false;
    {
      std::lock_guard<std::mutex> lk(hold_mu_);
      for (uint8_t h : t.holders[t.cur]) held = held || h;
    }
    if (held) {  // some client reads it in place: build the next version beside it
      t.cur = free_version(t);
      stats_.nr_apply_out_of_place++;
    }
    t.cur_published = false;
  }
  GP_CALL(gp_bucket_sum_into(t.versions[t.cur]->data(), in, ptrs.data(), (int)ptrs.size(),
                             t.row_count * ROW_DATA_SIZE, stream_));
  GP_CALL(gp_stream_synchronize(stream_));
  stats_.nr_apply_launches++;
  stats_.nr_buckets_applied += ptrs.size();
  t.pending.clear();  // releases oplog slices / staging buffers
  stats_.apply_time += now_s() - t0;
}

// TabletStorage::clock (src/server/tablet-server.cpp:169-212).
void TabletServer::clock(uint32_t client_id, iter_t clock, uint32_t table_id) {
  stats_.nr_clock++;
  GP_CHECK_LT(table_id, tables_.size());
  DataTable &t = tables_[table_id];
  GP_CHECK_LT(client_id, t.vec_clock.size());
  if (t.vec_clock[client_id] != INITIAL_DATA_AGE) GP_CHECK_EQ(clock, t.vec_clock[client_id] + 1);
  t.vec_clock[client_id] = clock;
  const iter_t new_global = *std::min_element(t.vec_clock.begin(), t.vec_clock.end());
  if (new_global != t.global_clock) {
    if (t.global_clock != INITIAL_DATA_AGE) GP_CHECK_EQ(new_global, t.global_clock + 1);
    t.global_clock = new_global;
    send_refresh(table_id);
  }
}

// process_multiclient_pending_reads (tablet-server.cpp:136-163): the whole
// shard to every client, starting client rotated by the clock.
void TabletServer::send_refresh(uint32_t table_id) {
  DataTable &t = tables_[table_id];
  apply_pending(t);
  const double t0 = now_s();
  const iter_t n = (iter_t)num_clients_;
  const uint32_t start = (uint32_t)(((t.global_clock % n) + n) % n);
  const int ver = t.row_count ? t.cur : -1;
  const float *rows = ver >= 0 ? t.versions[ver]->data() : nullptr;
  if (ver >= 0) t.cur_published = true;
  for (uint32_t i = 0; i < num_clients_; ++i) {
    const uint32_t c = (start + i) % num_clients_;
    RowBatchReply r{server_id_, t.global_clock, t.vec_clock[c], table_id,
                    t.row_keys.data(), rows, t.row_count, ver};
    // Record the hold before the client can release it (a same-node client's
    // release arrives on another thread as soon as the frame is out).
    if (ver >= 0) {
      std::lock_guard<std::mutex> lk(hold_mu_);
      t.holders[ver][c] = 1;
    }
    if (!sink_->read_row_batch_reply(c, r) && ver >= 0) {
      std::lock_guard<std::mutex> lk(hold_mu_);
      t.holders[ver][c] = 0;
    }
  }
  stats_.nr_refresh++;
  stats_.refresh_time += now_s() - t0;
}

}  // namespace geeps
