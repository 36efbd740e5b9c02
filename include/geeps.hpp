#ifndef __geeps_hpp__
#define __geeps_hpp__

// GeePS public API, served by the MI355X-native libgeeps
// (geeps_amd/csrc/geeps/).
//
// Drop-in for the reference's include/geeps.hpp:42-98 (cuihenggang/geeps):
// the GeePsConfig field order, types and defaults and every GeePs member
// function signature are unchanged, so apps/helloworld and apps/caffe compile
// and link against this library without edits.  Field-by-field layout parity
// with the reference header is tested in tests/test_layout.py.
//
// Behavioural notes relative to the reference:
//   * `port_list` is honoured (the reference never copies it into the client
//     library, src/client/clientlib.cpp:57-60, so two processes on one host
//     collide on tcp_base_port); an empty port_list keeps the reference
//     behaviour of tcp_base_port for every host.
//   * Update buffers handed out by PreUpdate live in device memory (HBM), as
//     in the reference (src/client/clientlib.cpp:522-565).

#include <string>
#include <vector>

#include "geeps-user-defined-types.hpp"

using std::string;
using std::vector;

struct GeePsConfig {
  uint num_tables;
  std::vector<std::string> host_list;
  std::vector<uint> port_list;
  uint tcp_base_port;
  uint num_comm_channels;
  std::string output_dir;
  iter_t log_interval;
  int pp_policy;
  int local_opt;
  size_t gpu_memory_capacity;
  // 0: no warning; 1: guarantee double buffering for the thread cache;
  // 2: all local data in GPU memory; 3: all parameter cache in GPU memory.
  int mm_warning_level;
  int pinned_cpu_memory;
  int read_my_writes;

  GeePsConfig()
      : num_tables(1),
        tcp_base_port(9090),
        num_comm_channels(1),
        output_dir(""),
        log_interval(0),
        pp_policy(0),
        local_opt(1),
        gpu_memory_capacity(std::numeric_limits<size_t>::max()),
        mm_warning_level(1),
        pinned_cpu_memory(1),
        read_my_writes(0) {}
};

class GeePs {
 public:
  GeePs(uint process_id, const GeePsConfig &config);
  void Shutdown();
  std::string GetStats();
  void StartIterations();

  // Virtual iteration: declare the access sequence of one clock.
  int VirtualRead(size_t table_id, const vector<size_t> &row_ids, int slack);
  int VirtualPostRead(int prestep_handle);
  int VirtualPreUpdate(size_t table_id, const vector<size_t> &row_ids);
  int VirtualUpdate(int prestep_handle);
  int VirtualLocalAccess(const vector<size_t> &row_ids, bool fetch);
  int VirtualPostLocalAccess(int prestep_handle, bool keep);
  int VirtualClock();
  void FinishVirtualIteration();

  // Real accesses, replaying the declared sequence.
  bool Read(int handle, RowData **buffer_ptr);
  void PostRead(int handle);
  void PreUpdate(int handle, RowOpVal **buffer_ptr);
  void Update(int handle);
  bool LocalAccess(int handle, RowData **buffer_ptr);
  void PostLocalAccess(int handle);
  void Clock();
};

#endif  // __geeps_hpp__
