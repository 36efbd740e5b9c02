// ClientLib's data path: Read / PostRead / PreUpdate / Update (HBM and host
// tier), the clock's push, the refresh into the param cache.  Reference:
// src/client/clientlib-data.cpp, clientlib-bg-access.cpp.
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
    if (op.host_run_channel >= 0) {
      // the op's rows are this channel's host rows [lo, +rows) in order: one
      // copy straight from the host cache, under the lock a refresh takes
      if ((int)ch.id != op.host_run_channel) continue;
      const size_t vals = std::min(op.num_vals_limit, op.rows.size() * ROW_DATA_SIZE);
      if (vals)
        GP_CALL(gp_memcpy_async(op.buffer.data(), pc.cpu.data->data() + op.host_run_lo * ROW_DATA_SIZE,
                                vals * sizeof(float), channels_[0]->stream->get()));
      channels_[0]->stream->sync();
      std::lock_guard<std::mutex> slk(stats_mu_);
      stats_.nr_read_host_run++;
      continue;
    }
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
  // Each row's first write of the clock is the fused init 0.0f + x when this
  // clock's host-tier update ops write every row once (the oplog is then
  // never zeroed)
  std::vector<uint8_t> fused(channels_.size(), 0);
  for (auto &chp : channels_) fused[chp->id] = started_ && chp->host_init_ok[pre.table_id];
  const int rc = pre.host_run_channel;
  if (rc >= 0 && fused[rc] && pre.num_vals_limit >= pre.rows.size() * ROW_DATA_SIZE) {
    // The op's rows are one channel's host rows [lo, +rows) in order: one copy
    // straight into the oplog.  It holds x where the init writes 0.0f + x;
    // they differ only for -0.0, and the server's sum from +0.0 makes both
    // +0.0 (the HBM tier's direct oplog).
    Channel &ch = *channels_[rc];
    std::shared_ptr<HostBuf> oplog;
    {
      std::lock_guard<std::mutex> lk(ch.mu);
      oplog = get_host_oplog(ch.tables[pre.table_id].cpu, clock, /*zero=*/false);
    }
    if (vals)
      GP_CALL(gp_memcpy_async(oplog->data() + pre.host_run_lo * ROW_DATA_SIZE, pre.buffer.data(),
                              vals * sizeof(float), ch0.stream->get()));
    ch0.stream->sync();
    std::lock_guard<std::mutex> lk(stats_mu_);
    stats_.nr_update_host_init++;
    stats_.nr_update_host_run++;
    return;
  }
  const size_t piece_vals = kHostPieceRows * ROW_DATA_SIZE;
  const size_t pieces = (vals + piece_vals - 1) / piece_vals;
  while (host_events_.size() < pieces) host_events_.push_back(std::make_unique<Event>());
  for (size_t k = 0; k < pieces; ++k) {
    const size_t f0 = k * piece_vals, f1 = std::min(vals, f0 + piece_vals);
    GP_CALL(gp_memcpy_async(cpu_buffer_.data() + f0, pre.buffer.data() + f0, (f1 - f0) * sizeof(float),
                            ch0.stream->get()));
    host_events_[k]->record(*ch0.stream);
  }
  // the clock's host oplogs (zeroed when new, unless fused) while the rows
  // come down
  std::vector<std::shared_ptr<HostBuf>> oplogs(channels_.size());
  for (auto &chp : channels_) {
    std::lock_guard<std::mutex> lk(chp->mu);
    HostTier &cpu = chp->tables[pre.table_id].cpu;
    if (cpu.num_rows) oplogs[chp->id] = get_host_oplog(cpu, clock, /*zero=*/!fused[chp->id]);
  }
  if (std::find(fused.begin(), fused.end(), 1) != fused.end()) {
    std::lock_guard<std::mutex> lk(stats_mu_);
    stats_.nr_update_host_init++;
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
      GP_CALL((fused[ch.id] ? gp_host_scatter_init_rows : gp_host_scatter_add_rows)(
          oplogs[ch.id]->data(), cpu_buffer_.data(), idx + e.first, e.second - e.first, gp_double_index{0, 0},
          ROW_DATA_SIZE, pre.num_vals_limit));
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
std::shared_ptr<HostBuf> ClientLib::get_host_oplog(HostTier &cpu, iter_t clock, bool zero) {
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
  if (zero) buf->zero();
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
                    << oplog->bytes() << ": " << ipc_describe(ref.handle) << "\n";
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

}  // namespace geeps
