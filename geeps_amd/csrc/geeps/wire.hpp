#ifndef GEEPS_AMD_WIRE_HPP_
#define GEEPS_AMD_WIRE_HPP_

/*
 * The message structs below restate GeePS's wire protocol
 * (cuihenggang/geeps, src/common/wire-protocol.hpp), whose layout they must
 * keep byte-for-byte.  The upstream notice for that protocol:
 *
 * Copyright (c) 2016, Carnegie Mellon University.
 * All rights reserved.
 *
 * Redistribution and use in source and binary forms, with or without
 * modification, are permitted provided that the following conditions
 * are met:
 * 1. Redistributions of source code must retain the above copyright
 *    notice, this list of conditions and the following disclaimer.
 * 2. Redistributions in binary form must reproduce the above copyright
 *    notice, this list of conditions and the following disclaimer in the
 *    documentation and/or other materials provided with the distribution.
 * 3. Neither the name of the University nor the names of its contributors
 *    may be used to endorse or promote products derived from this software
 *    without specific prior written permission.
 *
 * THIS SOFTWARE IS PROVIDED BY THE COPYRIGHT HOLDERS AND CONTRIBUTORS
 * ``AS IS'' AND ANY EXPRESS OR IMPLIED WARRANTIES, INCLUDING, BUT NOT
 * LIMITED TO, THE IMPLIED WARRANTIES OF MERCHANTABILITY AND FITNESS FOR
 * A PARTICULAR PURPOSE ARE DISCLAIMED.  IN NO EVENT SHALL THE COPYRIGHT
 * HOLDERS OR CONTRIBUTORS BE LIABLE FOR ANY DIRECT, INDIRECT,
 * INCIDENTAL, SPECIAL, EXEMPLARY, OR CONSEQUENTIAL DAMAGES (INCLUDING,
 * BUT NOT LIMITED TO, PROCUREMENT OF SUBSTITUTE GOODS OR SERVICES; LOSS
 * OF USE, DATA, OR PROFITS; OR BUSINESS INTERRUPTION) HOWEVER CAUSED
 * AND ON ANY THEORY OF LIABILITY, WHETHER IN CONTRACT, STRICT
 * LIABILITY, OR TORT (INCLUDING NEGLIGENCE OR OTHERWISE) ARISING IN ANY
 * WAY OUT OF THE USE OF THIS SOFTWARE, EVEN IF ADVISED OF THE
 * POSSIBILITY OF SUCH DAMAGE.
 */

// Wire layout of the update push and the shard refresh (the two ends of the
// reduction path).  Byte-compatible with the reference's
// src/common/wire-protocol.hpp:42-131 so that frames produced by either side
// decode on the other: the 24-byte headers, RowKey (16 B) and the Command
// numbering are identical (checked by tests/test_layout.py).
//
// A CLOCK_WITH_UPDATES_BATCH frame is [header][RowKey x n][RowOpVal x n]
// (src/client/encoder-decoder.cpp:105-150); a READ_ROW_BATCH reply is
// [sc_read_row_batch_msg_t][RowKey x n][RowData x n]
// (src/server/server-encoder-decoder.cpp:228-250).

#include <stdint.h>

#include <vector>

#include "geeps-user-defined-types.hpp"
#include "gp_reduce.h"
#include "hostshare.hpp"

// Clock value of a table nobody has clocked yet, and the largest clock
// (src/common/internal-config.hpp:34-36).
#define BIG_ITER 10000000
#define MAX_CLOCK BIG_ITER
#define INITIAL_DATA_AGE -BIG_ITER

enum Command {
  FIND_ROW,
  READ_ROW_BATCH,
  CLOCK,
  CLOCK_WITH_UPDATES_BATCH,
  ADD_ACCESS_INFO,
  GET_STATS,
  SHUTDOWN
};

struct RowKey {
  table_id_t table;
  row_idx_t row;
  RowKey(table_id_t t = 0, row_idx_t r = 0) : table(t), row(r) {}
};
typedef std::vector<RowKey> RowKeys;

// client -> server: one clock's summed deltas for the server's row range.
struct cs_clock_with_updates_batch_msg_t {
  command_t cmd;
  uint32_t client_id;
  iter_t clock;
  uint32_t table_id;
  int update_branch_id;
  int read_branch_id;
};

// client -> server: clock with no updates.
struct cs_clock_msg_t {
  command_t cmd;
  uint32_t client_id;
  iter_t clock;
  uint32_t table_id;
  int read_branch_id;
};

// server -> client: the refreshed shard.
struct sc_read_row_batch_msg_t {
  command_t cmd;
  uint32_t server_id;
  iter_t data_age;
  iter_t self_clock;
  uint32_t table_id;
  int branch_id;
};

// ---------------------------------------------------------------------------
// libgeeps-internal frames for same-node peers (not part of the reference
// protocol; numbered clear of its Command enum).  Bulk rows move device to
// device (xGMI between MI355X GPUs, or within one GPU) through IPC-mapped
// HBM; TCP carries only these small control frames.
// ---------------------------------------------------------------------------
constexpr command_t kCmdRefreshAck = 101;  // client -> server: master version released
// client -> server, the last frame on a connection: the client's reader has
// handled the server's SHUTDOWN and every frame before it (each version handle
// they named is mapped), and no device work of the client still reads the
// server's memory.  The server's process outlives this: a handle opened after
// its exporter exited is refused ("Invalid IPC handle ... and 0").
constexpr command_t kCmdReaderDone = 102;
constexpr uint32_t kIpcHandleBytes = GP_IPC_HANDLE_BYTES;  // the C-ABI's opaque handle

// 4th part of a CLOCK_WITH_UPDATES_BATCH whose rows stay in the client's oplog.
// The RowKey part is sent on the first such message per (server, table) only:
// the server takes the shard's keys from its first message and sums later ones
// positionally (tablet-server.cpp:108-116), so later messages carry an empty
// key part and the row count is bytes / sizeof(RowData).
struct IpcRowsRef {
  uint64_t buffer_id;   // (table << 32) | oplog pool index: stable, unique per client
  uint64_t offset;      // bytes from the buffer base to this server's slice
  uint64_t bytes;
  uint32_t has_handle;  // first use of buffer_id: `handle` is valid
  uint32_t pad;
  uint8_t handle[kIpcHandleBytes];
};

// 5th part of a CLOCK_WITH_UPDATES_BATCH from a same-node client of a table
// with a host tier (round 5): the host-tier rows stay in the client's host
// oplog too, shared memory the server maps (hostshare.hpp), and part 2 is
// empty.  The handle rides along on the first use of buffer_id per server.
struct HostRowsRef {
  uint64_t buffer_id;   // (table << 32) | host oplog pool index
  uint64_t offset;      // bytes from the buffer base to this server's host-tier rows
  uint64_t bytes;
  uint32_t has_handle;  // first use of buffer_id: `handle` is valid
  uint32_t pad;
  geeps::HostShareHandle handle;
};

// 4th part of a READ_ROW_BATCH from a same-node server: the shard is the
// server's master version `version`, which the client reads in place through
// the IPC mapping of that version's buffer (the handle rides along the first
// time a version is named to this client) until a later refresh replaces it.
struct IpcRefreshVersion {
  int32_t version;
  uint32_t has_handle;
  uint64_t num_rows;
  uint8_t handle[kIpcHandleBytes];
};

// The client no longer reads master version `version` of `table_id` in place.
struct RefreshAckMsg {
  command_t cmd;
  uint32_t client_id;
  uint32_t table_id;
  int32_t version;
};

// IPC recovery.  A handle the runtime refuses to map, or a
// mapping without the exporter's tag, costs one resend of the rows over the
// socket instead of the job:
//
// server -> client: the server could not map the oplog buffer that the
// client's CLOCK_WITH_UPDATES_BATCH for (table, clock) named.  The client
// sends that slice again as an ordinary socket frame (keys + rows), and
// exports a fresh buffer in place of this one on its next use.  The server's
// reader holds the client's later frames back until the resend arrives, so
// the server sees the client's messages in their order.
constexpr command_t kCmdOplogNack = 103;
// `unmapped`: kNackDevice, the HBM slice's buffer (replaced on its next use);
// kNackHost, the host-tier rows' shared buffer (the client's frames to this
// server then carry those rows again).
constexpr uint32_t kNackDevice = 1, kNackHost = 2;
struct OplogNackMsg {
  command_t cmd;
  uint32_t server_id;
  uint32_t table_id;
  uint32_t unmapped;
  iter_t clock;
  uint64_t buffer_id;
};
// client -> server: the client could not map master version `version` of
// `table_id` that the refresh of data age `data_age` named.  The server sends
// that refresh again as a socket frame (keys + rows of the version, which the
// client still holds, so it is unchanged), takes the hold back and forgets the
// handle went out (the next refresh naming the version sends it again).  The
// client's reader holds later frames back until the resend arrives.
constexpr command_t kCmdVersionNack = 104;
struct VersionNackMsg {
  command_t cmd;
  uint32_t client_id;
  uint32_t table_id;
  int32_t version;
  iter_t data_age;
  iter_t self_clock;
};

#endif  // GEEPS_AMD_WIRE_HPP_
