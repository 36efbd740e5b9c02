// layout_probe.cpp — prints the byte layout of the types that cross the
// gradient-update path's boundaries (row values, row keys, wire headers,
// GeePsConfig) as one JSON object.
//
// TEST INFRASTRUCTURE ONLY.  oracle/Makefile compiles it twice:
//   -DPROBE_REF : against the reference's own, unmodified, self-contained
//                 headers under /root/reference (include/geeps.hpp,
//                 include/geeps-user-defined-types.hpp,
//                 src/common/wire-protocol.hpp, src/common/internal-config.hpp)
//                 -> oracle/_ref/layout_probe (never committed);
//   (default)   : against this repo's drop-in headers (include/) and
//                 libgeeps' wire header -> oracle/build/layout_probe_ours.
// tests/test_layout.py requires the two outputs to be identical; the
// reference output is also frozen in tests/golden/ref_layout.json (made by
// tests/golden/make_golden.py) so the check runs where /root/reference is
// absent.
#include <cstddef>
#include <cstdio>

#ifdef PROBE_REF
#include "geeps.hpp"
#include "common/internal-config.hpp"
#include "common/wire-protocol.hpp"
#else
#include "geeps.hpp"
#include "wire.hpp"
#endif

#define FIELD(T, f) std::printf("  \"" #T "." #f "\": [%zu, %zu],\n", offsetof(T, f), sizeof(((T *)0)->f))
#define SIZE(T) std::printf("  \"sizeof(" #T ")\": %zu,\n", sizeof(T))

#pragma GCC diagnostic ignored "-Winvalid-offsetof"

int main() {
  std::printf("{\n");
  SIZE(ArrayData);
  SIZE(RowData);
  SIZE(RowOpVal);
  SIZE(val_t);
  SIZE(row_idx_t);
  SIZE(table_id_t);
  SIZE(iter_t);
  SIZE(command_t);
  std::printf("  \"ROW_DATA_SIZE\": %d,\n", (int)ROW_DATA_SIZE);
  std::printf("  \"INITIAL_DATA_AGE\": %d,\n", (int)INITIAL_DATA_AGE);
  std::printf("  \"MAX_CLOCK\": %d,\n", (int)MAX_CLOCK);
  SIZE(RowKey);
  FIELD(RowKey, table);
  FIELD(RowKey, row);
  std::printf("  \"Command\": [%d, %d, %d, %d, %d, %d, %d],\n", (int)FIND_ROW,
              (int)READ_ROW_BATCH, (int)CLOCK, (int)CLOCK_WITH_UPDATES_BATCH,
              (int)ADD_ACCESS_INFO, (int)GET_STATS, (int)SHUTDOWN);
  SIZE(cs_clock_msg_t);
  FIELD(cs_clock_msg_t, cmd);
  FIELD(cs_clock_msg_t, client_id);
  FIELD(cs_clock_msg_t, clock);
  FIELD(cs_clock_msg_t, table_id);
  FIELD(cs_clock_msg_t, read_branch_id);
  SIZE(cs_clock_with_updates_batch_msg_t);
  FIELD(cs_clock_with_updates_batch_msg_t, cmd);
  FIELD(cs_clock_with_updates_batch_msg_t, client_id);
  FIELD(cs_clock_with_updates_batch_msg_t, clock);
  FIELD(cs_clock_with_updates_batch_msg_t, table_id);
  FIELD(cs_clock_with_updates_batch_msg_t, update_branch_id);
  FIELD(cs_clock_with_updates_batch_msg_t, read_branch_id);
  SIZE(sc_read_row_batch_msg_t);
  FIELD(sc_read_row_batch_msg_t, cmd);
  FIELD(sc_read_row_batch_msg_t, server_id);
  FIELD(sc_read_row_batch_msg_t, data_age);
  FIELD(sc_read_row_batch_msg_t, self_clock);
  FIELD(sc_read_row_batch_msg_t, table_id);
  FIELD(sc_read_row_batch_msg_t, branch_id);
  SIZE(GeePsConfig);
  FIELD(GeePsConfig, num_tables);
  FIELD(GeePsConfig, host_list);
  FIELD(GeePsConfig, port_list);
  FIELD(GeePsConfig, tcp_base_port);
  FIELD(GeePsConfig, num_comm_channels);
  FIELD(GeePsConfig, output_dir);
  FIELD(GeePsConfig, log_interval);
  FIELD(GeePsConfig, pp_policy);
  FIELD(GeePsConfig, local_opt);
  FIELD(GeePsConfig, gpu_memory_capacity);
  FIELD(GeePsConfig, mm_warning_level);
  FIELD(GeePsConfig, pinned_cpu_memory);
  FIELD(GeePsConfig, read_my_writes);
  {
    GeePsConfig c;  // defaults (include/geeps.hpp:60-70)
    std::printf("  \"GeePsConfig.defaults\": [%u, %u, %u, %d, %d, %d, %zu, %d, %d, %d],\n",
                c.num_tables, c.tcp_base_port, c.num_comm_channels,
                (int)c.log_interval, c.pp_policy, c.local_opt,
                c.gpu_memory_capacity, c.mm_warning_level, c.pinned_cpu_memory,
                c.read_my_writes);
  }
  {
    ArrayData a;  // ArrayData() zero-initialises (geeps-user-defined-types.hpp:56-64)
    int zero = 1;
    for (int i = 0; i < ROW_DATA_SIZE; ++i) zero &= (a.data[i] == 0.0f);
    std::printf("  \"ArrayData.zero_init\": %d\n", zero);
  }
  std::printf("}\n");
  return 0;
}
