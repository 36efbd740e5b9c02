// ClientLib's virtual iteration: the op sequence, the param cache placement
// (HBM / host tier), the DoubleIndexes and plans.  Reference:
// src/client/clientlib-viter.cpp.
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
    ch.host_init_ok.assign(config_.num_tables, false);
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
      // The host tier's oplog, likewise from its own (host-tier) update ops.
      // Not with read-my-writes: a host-tier Update adds piece by piece, each
      // under the channel lock, so a refresh between pieces would re-apply
      // rows not yet written this clock.
      std::vector<uint8_t> hseen(pc.cpu.num_rows, 0);
      size_t hcovered = 0;
      bool hok = pc.cpu.num_rows > 0 && !config_.read_my_writes;
      for (size_t i = 0; i < end && hok; ++i) {
        const OpInfo &w = opseq_[i];
        if (w.type != OpInfo::WRITE || w.local || w.table_id != t || !w.cpu) continue;
        const OpInfo &pre = opseq_[w.prestep_handle];
        if (pre.num_vals_limit < pre.rows.size() * ROW_DATA_SIZE) hok = false;
        for (row_idx_t r : pre.rows) {
          if (channel_of(t, r) != ch.id) continue;
          if (hseen[pc.cpu.index.at(r)]++) hok = false;
          ++hcovered;
        }
      }
      ch.host_init_ok[t] = hok && hcovered == pc.cpu.num_rows;
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
    // row_index_cpu, clientlib-viter.cpp:853-876); no device index or plans.
    // Its rows one channel's host cache rows in order (op row j -> host row
    // lo + j): its Read and Update copy them whole (read_batch_host)
    op.direct_channel = -1;
    op.host_run_channel = -1;
    for (uint32_t c = 0; c < num_channels_ && host_runs_; ++c) {
      if (per[c].size() != op.rows.size() || op.rows.empty()) continue;
      bool run = true;
      for (size_t j = 0; j < per[c].size() && run; ++j)
        run = per[c][j].id0 == j && per[c][j].id1 == per[c][0].id1 + j;
      if (run) {
        op.host_run_channel = (int)c;
        op.host_run_lo = per[c][0].id1;
      }
    }
    op.host_index = std::move(flat);
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

}  // namespace geeps
