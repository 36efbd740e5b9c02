#ifndef GEEPS_AMD_SERVER_HPP_
#define GEEPS_AMD_SERVER_HPP_

// Tablet server: the server half of the gradient-update reduction path.
//
// One TabletServer runs per (process, communication channel), as the
// reference's ServerThreadEntry does (src/server/server-entry.cpp:51-88).  It
// owns, per table, the master copy of this server's row shard in HBM and the
// vector clock of its clients, and serves two messages:
//
//   CLOCK_WITH_UPDATES_BATCH  -> update_row_batch() then clock()
//                                (ClientServerDecode::clock_with_updates_batch,
//                                 src/server/server-encoder-decoder.cpp:86-113)
//   CLOCK                     -> clock()
//
// The reference adds every arriving update into the CPU master immediately
// (TabletStorage::apply_updates -> cpu_add, src/server/tablet-server.cpp:119-134).
// Here arriving update batches queue as device buckets in arrival order and
// are summed into the master by ONE bucket-sum launch right before the master
// is observed (the refresh sent when the global clock advances), or when the
// queue reaches kMaxPendingBuckets.  The per-element order of fp32 adds is the
// arrival order in both cases, so the master is bit-identical to the
// reference's; the device reads each bucket once and the master once per
// refresh instead of once per client.
//
// Versions.  The reference replies a COPY of the shard to every client
// (server-encoder-decoder.cpp:228-250).  Here a refresh publishes the current
// master version, and same-process / same-node clients read it in place (over
// IPC-mapped HBM) until a later refresh replaces it; they release it then.  A
// published version is never written again while any client holds it: the
// next apply writes a new version out of place (gp_bucket_sum_into: same
// bytes as the in-place sum), into a version no client holds, allocating one
// when none is free, up to clients + 2 versions.  A client is marked as
// holding a version when the refresh is SENT, and gives the one before back
// when its reader thread TAKES the next refresh, so under SSP a lagging reader
// can hold several (up to slack + 2).  When every version is held and the cap
// is reached, the apply waits for a release.  Releases arrive on the socket
// reader threads (or inside this thread for the in-process client, which
// holds only the current version), each the reader catching up on refreshes
// already sent -- progress that needs nothing from this thread -- except for
// direct Reads (GEEPS_DIRECT_READ=1): a version a direct Read pins when a
// refresh replaces it goes back only at the app thread's PostRead, and that
// thread may be blocked in a Read of another table waiting on this very
// server.  A client therefore keeps at most ONE such deferred version per
// (server, table) -- a Read that would pin a second one gathers instead
// (client_data.cpp, read_batch).  Of the clients + 1 versions other than the one
// being replaced, at most `clients` are then deferred, so at least one is free
// or held only by readers that will catch up: the wait always ends.

#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "device.hpp"
#include "wire.hpp"

namespace geeps {

// Rows of one client's clock update for one server: n keys and n RowOpVal.
// Exactly one of `device_rows` or `host_rows` (received from a socket into
// pinned memory) is set.  `device_rows` is the in-process client's oplog slice
// (kept alive by `keepalive` until applied) or a same-node peer's oplog slice
// through an IPC mapping, which the sum reads in place when the peer is on
// this GPU; with `stage` (the peer is on another GPU) it is first copied into
// local HBM on the server's copy stream, so the sum reads only local HBM.  The
// peer's buffer stays valid either way: it reclaims an oplog only once every
// server's refresh covers its clock, and a refresh leaves a server only after
// its apply consumed the bucket.
struct UpdateBatch {
  uint32_t client_id = 0;
  iter_t clock = 0;
  uint32_t table_id = 0;
  // n keys at `keys`, kept alive by `keys_owner` (the client's immutable
  // param-cache key list, or the received frame's copy): never copied per push.
  const RowKey *keys = nullptr;
  size_t num_rows = 0;
  std::shared_ptr<const void> keys_owner;
  const float *device_rows = nullptr;
  bool stage = false;
  std::shared_ptr<void> keepalive;
  std::shared_ptr<PinnedArray<float>> host_rows;
  // The in-process client's batch of a table with a host tier: its first
  // `split` rows are host-tier rows at `host_head` (its host oplog, kept alive
  // by head_keepalive), the other num_rows - split at `device_rows`.  The
  // server stages the two into one bucket in HBM.
  size_t split = 0;
  const float *host_head = nullptr;
  std::shared_ptr<const void> head_keepalive;
};

// The refreshed shard, as the server hands it to a client sink.  `device_rows`
// is master version `version` (-1: no rows yet).  It stays valid after the
// sink call only if the sink reports that the client holds it; the client
// then gives it back through TabletServer::release().
struct RowBatchReply {
  uint32_t server_id;
  iter_t data_age;
  iter_t self_clock;
  uint32_t table_id;
  const RowKey *keys;
  const float *device_rows;
  size_t num_rows;
  int version;
};

// Where the server sends refreshed shards (ServerClientEncode::read_row_batch_reply,
// src/server/server-encoder-decoder.cpp:228-250).
class ClientSink {
 public:
  virtual ~ClientSink() = default;
  // Returns true if the client keeps reading reply.device_rows after the call
  // (it will release reply.version).
  virtual bool read_row_batch_reply(uint32_t client_id, const RowBatchReply &reply) = 0;
  // Every client has said SHUTDOWN: nothing more will be sent to `client_id`.
  virtual void shutdown_ack(uint32_t client_id) = 0;
};

struct ServerStats {
  uint64_t nr_update = 0;        // rows received (tablet-server.hpp stats)
  uint64_t nr_local_update = 0;
  uint64_t nr_clock = 0;
  uint64_t nr_refresh = 0;
  uint64_t nr_apply_launches = 0;
  uint64_t nr_apply_out_of_place = 0;  // applies that built a new master version
  uint64_t nr_buckets_applied = 0;
  uint64_t nr_versions = 0;            // master versions allocated (all tables)
  double apply_time = 0;         // s, including the launch sync
  double stage_time = 0;         // s, H2D of socket-delivered buckets (host side)
  uint64_t nr_peer_staged = 0;   // buckets copied in from a peer GPU before the sum
  double version_wait_time = 0;  // s, applies waiting for a master version release
  double refresh_time = 0;       // s, sending refreshed shards
  std::string to_json() const;
};

class TabletServer {
 public:
  static constexpr size_t kMaxPendingBuckets = 8;

  // `device`: the HIP device the owning process works on.  The server thread
  // selects it before its first HIP call, so the master shard, the staging
  // buffers and every launch land on that GPU (a new thread starts on device 0).
  // `stream`: the HIP stream all of this server's device work goes to (not
  // owned; the channel's service stream).
  TabletServer(uint32_t server_id, uint32_t channel_id, uint32_t num_clients,
               uint32_t num_tables, ClientSink *sink, int device, gp_stream stream);
  ~TabletServer();
  TabletServer(const TabletServer &) = delete;
  TabletServer &operator=(const TabletServer &) = delete;

  // Thread-safe; processed in posting order by the server thread.
  void post_updates(UpdateBatch &&batch);
  void post_clock(uint32_t client_id, iter_t clock, uint32_t table_id);
  // Client `client_id` will send nothing more.  Once every client has said so,
  // each is acknowledged through ClientSink::shutdown_ack.
  void post_shutdown(uint32_t client_id);
  // Client `client_id` no longer reads master version `version` of table
  // `table_id` in place.  Thread-safe; any thread.
  void release(uint32_t client_id, uint32_t table_id, int version);
  // ... nor any version of any table (its SHUTDOWN arrived).
  void release_all(uint32_t client_id);
  // Master version `version` of `table_id`, which `client_id` holds (so the
  // server does not write it): its rows, row count and keys, for a resend of
  // a refresh the client could not map (kCmdVersionNack).  Thread-safe.
  void held_version(uint32_t client_id, uint32_t table_id, int version, const float **rows,
                    size_t *num_rows, const RowKey **keys);
  // Blocks until every client has sent SHUTDOWN and all were acknowledged.
  void wait_shutdown();
  // Blocks until every message posted before it has been processed.
  void drain();
  void stop();
  std::string stats_json();

  uint32_t server_id() const { return server_id_; }

 private:
  struct Pending {
    const float *rows;
    std::shared_ptr<void> keepalive;
    std::shared_ptr<Event> staged;  // a peer copy into `rows` on copy_streams_[client]
  };
  struct DataTable {
    std::vector<iter_t> vec_clock;
    iter_t global_clock = INITIAL_DATA_AGE;
    size_t row_count = 0;
    std::vector<RowKey> row_keys;
    // master versions; `cur` is the latest, `cur_published` once a refresh
    // has handed it out (from then on it is only read)
    std::vector<std::unique_ptr<DeviceArray<float>>> versions;
    int cur = -1;
    bool cur_published = false;
    // [version][client]: the client reads that version in place (hold_mu_)
    std::vector<std::vector<uint8_t>> holders;
    std::vector<Pending> pending;
    std::vector<std::shared_ptr<DeviceArray<float>>> stage_pool;
  };
  struct Msg {
    enum Kind { kUpdates, kClock, kShutdown, kDrain, kStop } kind;
    UpdateBatch batch;
    uint32_t client_id = 0;
    iter_t clock = 0;
    uint32_t table_id = 0;
    std::function<void()> done;
  };

  void run();
  void update_row_batch(UpdateBatch &batch);
  void clock(uint32_t client_id, iter_t clock, uint32_t table_id);
  void apply_pending(DataTable &t);
  void send_refresh(uint32_t table_id);
  std::shared_ptr<DeviceArray<float>> stage_buffer(DataTable &t);
  int free_version(DataTable &t);

  const uint32_t server_id_, channel_id_, num_clients_;
  ClientSink *sink_;
  const int device_;
  std::vector<DataTable> tables_;
  const gp_stream stream_;
  ServerStats stats_;

  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Msg> queue_;
  std::mutex hold_mu_;  // DataTable::holders (and the versions vector's size)
  std::condition_variable release_cv_;  // a hold ended (release / release_all)
  uint64_t releases_ = 0;               // holds ended so far (hold_mu_): reader progress
  // peer copies of other GPUs' buckets: one stream per client (made on first
  // use, server thread only), so slices from different peers come over their
  // own xGMI links at once instead of one after another on a single stream
  std::vector<std::unique_ptr<Stream>> copy_streams_;
  uint32_t shutdown_count_ = 0;  // server thread only
  bool shutdown_done_ = false;    // guarded by mu_
  std::condition_variable shutdown_cv_;
  std::thread thread_;
};

}  // namespace geeps

#endif  // GEEPS_AMD_SERVER_HPP_
