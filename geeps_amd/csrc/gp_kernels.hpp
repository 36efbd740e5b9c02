#ifndef GP_KERNELS_HPP_
#define GP_KERNELS_HPP_

// gp_kernels.hpp — the kernels of libgp_reduce and their launch logic, shared by
// its two kernel translation units: gp_reduce.hip (row plans, the bucket sums'
// C-ABI) and gp_unplanned.hip (the unplanned calls' device planning and plan
// cache).  Internal: not part of the C-ABI (include/gp_reduce.h).  Everything
// here is in an anonymous namespace, instantiated per translation unit; the
// thread's error message is one (gp_internal::set_error, gp_reduce.hip).
//
//  * bucket_sum_*_kernel — the server's N-way sum of client delta buckets into
//    the master shard (tablet-server.cpp:119-134), and the dense runs of the
//    row plans (1 bucket, the zero-input form, the NB = 0 copy).
//  * row_op_kernel / row_wave_kernel / row_op_seg_kernel — the row-indexed
//    scatter-add / gather / scatter-assign over a DoubleIndex
//    (row-op-util.cu:39-142).

#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "gp_reduce.h"

namespace gp_internal {
int set_error(int code, const char *msg);  // gp_reduce.hip
}

namespace {

typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kBlock = 256;
// A block-stride grid of this many blocks per CU saturates HBM on 256 CUs
// while keeping launch cost flat for any problem size.
constexpr int kBlocksPerCU = 8;
constexpr int kMaxBucketsPerLaunch = 8;

// the calling thread's gp_last_error message (one per process: gp_reduce.hip)
inline int set_error(int code, const std::string &msg) { return gp_internal::set_error(code, msg.c_str()); }

#define GP_HIP_TRY(expr)                                                    \
  do {                                                                      \
    hipError_t e_ = (expr);                                                 \
    if (e_ != hipSuccess) {                                                 \
      /* the runtime keeps a failed call's error as the thread's last   */ \
      /* error: clear it, or the next launch's hipGetLastError() check  */ \
      /* reports it (a refused IPC export failed a later sum, round 5)  */ \
      (void)hipGetLastError();                                              \
      return set_error(GP_ERR_HIP, std::string(#expr) + ": " +             \
                                       hipGetErrorString(e_));             \
    }                                                                       \
  } while (0)

// CU count per device, cached on first use and never reset: a device's CU
// count is fixed, and libgeeps' server, reader and app threads plan launches
// concurrently (the sweep kernel's grid must equal the plan's G), so nothing
// may zero a slot another thread reads.  Devices past kMaxDevices (or a failed
// query, e.g. no GPU in a CPU-only test) read 256, the MI355X count.
constexpr int kMaxDevices = 64;
std::atomic<int> g_num_cus[kMaxDevices];  // zero-initialised (static storage)

inline int num_cus() {
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return 256;
  const int cached = g_num_cus[dev].load(std::memory_order_relaxed);
  if (cached > 0) return cached;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus <= 0)
    cus = 256;
  g_num_cus[dev].store(cus, std::memory_order_relaxed);
  return cus;
}

inline size_t grid_cap() { return (size_t)num_cus() * kBlocksPerCU; }

inline bool aligned16(const void *p) {
  return (reinterpret_cast<uintptr_t>(p) & 15u) == 0;
}

// ---------------------------------------------------------------------------
// N-way bucket sum: out[i] = ((in[i] + b0[i]) + b1[i]) + ... + b{NB-1}[i]
// ---------------------------------------------------------------------------

struct BucketPtrs {
  const float *p[kMaxBucketsPerLaunch];
};

// A launch that runs or exits at its start by a device word an earlier launch
// on the same stream wrote: the unplanned calls' steady state ("Device-built
// plans", gp_unplanned.hip) launches both the cached plan and the op-order
// fallback right behind the index check, and exactly one of them does any
// work, with no host round trip.  `word` holds the generation of the last call
// whose check found the index changed; this call's generation is `gen`.  A kernel's GATED = true
// instantiation runs this test first and takes the Gate as its last argument;
// GATED = false (the default, every other launch) compiles to the same code as
// without it (tests/test_kernel_schedule.py checks the sweep kernel's schedule).
// kGateIfSame: run only if the word does not hold this call's generation (the
// index is unchanged, the inverse map is sound); kGateIfChanged: only if it
// does.  kGateSelect (row kernels): always run -- on the launch's own rows
// (the cached sorted residual or inverse map) if unchanged, else on `alt` (the
// call's own index, its offsets, in op order): one launch serves both.
// `inv` (row_wave_kernel only): the launch walks destination rows 0 ..
// num_rows - 1 through an inverse map, inv[to] = entry << 32 | from, ~0 = no
// row (the unplanned calls' inverse plan), instead of reading `index`.
enum GateMode : unsigned { kGateIfSame = 0, kGateIfChanged = 1, kGateSelect = 2 };
struct Gate {
  const unsigned *word;
  unsigned gen;
  unsigned mode;
  const gp_double_index *alt;
  size_t alt_rows;
  uint64_t alt_off0, alt_off1;
  const uint64_t *inv;
};

// The gate word was written by an earlier launch on the stream and no kernel
// writes it while a gated one runs, so it is read as constant memory: a
// scalar load through the scalar cache (invalidated at every kernel start),
// not a system-coherent vector load that goes out to memory -- the first
// thing every block of a gated launch waits for (the steady state of a
// dense-run index is ~43 gated sweep launches).
__device__ __forceinline__ bool gate_changed(const Gate &g) {
  typedef const __attribute__((address_space(4))) unsigned CU;
  return *(CU *)(g.word) == g.gen;  // block-uniform (C-style: an address-space cast)
}

__device__ __forceinline__ bool gate_closed(const Gate &g) {
  // bitwise, so the mode, word pointer and generation load together (one
  // round trip, then the word's)
  const bool changed = gate_changed(g);
  return (g.mode != kGateSelect) & ((g.mode == kGateIfSame) == changed);
}

// A row kernel's GATED prologue: exit, or (select) switch to the alternative
// index when the check found the call's index changed.
#define GP_ROW_GATE(gate, index, num_rows, off0, off1)  \
  do {                                                  \
    if (gate.mode == kGateSelect) {                     \
      if (gate_changed(gate)) {                         \
        index = gate.alt;                               \
        num_rows = gate.alt_rows;                       \
        off0 = gate.alt_off0;                           \
        off1 = gate.alt_off1;                           \
      }                                                 \
    } else if (gate_closed(gate)) {                     \
      return;                                           \
    }                                                   \
  } while (0)

// hipLaunchKernelGGL of kernel K, or of its GATED form GK with *g last.  C:
// a compile-time condition for instantiating GK at all (only the forms the
// unplanned calls' steady state launches have gated twins).
#define GP_LAUNCH_GATED(C, g, K, GK, grid, block, s, ...)                 \
  do {                                                                    \
    if constexpr (C) {                                                    \
      if (g) {                                                            \
        hipLaunchKernelGGL(GK, grid, block, 0, s, __VA_ARGS__, *(g));     \
        break;                                                            \
      }                                                                   \
    }                                                                     \
    hipLaunchKernelGGL(K, grid, block, 0, s, __VA_ARGS__, Gate{});       \
  } while (0)

__device__ __forceinline__ f4 ld_stream(const f4 *p) {
  // Each bucket byte is read exactly once: non-temporal keeps the stream
  // from evicting anything useful from L2 / Infinity Cache.
  return __builtin_nontemporal_load(p);
}

// UNROLL consecutive block-strides per thread: (NB + 1) * UNROLL independent
// 16-B loads are in flight per lane before the first add.  ZIN (every form
// below has it): `in` is not read and the sum starts from +0.0f, so
// out = 0.0f + b0 -- the fused zerofy + scatter-add of a row plan's dense run
// (gp_scatter_init_rows_planned; 0.0f + -0.0f = +0.0f as after a memset).
template <int NB, int UNROLL, bool ZIN = false, bool GATED = false>
__global__ __launch_bounds__(kBlock) void bucket_sum_vec_kernel(
    f4 *__restrict__ out, const f4 *__restrict__ in, BucketPtrs b, size_t n4, Gate gate = Gate{}) {
  if constexpr (GATED) {
    if (gate_closed(gate)) return;
  }
  const size_t tile = (size_t)kBlock * UNROLL;
  const size_t stride = (size_t)gridDim.x * tile;
  const f4 *bp[NB > 0 ? NB : 1];  // NB = 0: a plain copy out = in (a gather plan's dense runs)
#pragma unroll
  for (int k = 0; k < NB; ++k) bp[k] = reinterpret_cast<const f4 *>(b.p[k]);

  size_t base = (size_t)blockIdx.x * tile + threadIdx.x;
  // Full tiles: no bounds checks inside.
  for (; base + (UNROLL - 1) * kBlock < n4; base += stride) {
    f4 acc[UNROLL];
    f4 v[NB > 0 ? NB : 1][UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) acc[u] = ZIN ? f4(0.0f) : in[base + u * kBlock];
#pragma unroll
    for (int k = 0; k < NB; ++k)
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) v[k][u] = ld_stream(bp[k] + base + u * kBlock);
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
#pragma unroll
      for (int k = 0; k < NB; ++k) acc[u] += v[k][u];  // bucket order 0..NB-1
      out[base + u * kBlock] = acc[u];
    }
  }
  // Ragged last tile.
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) {
    const size_t i = base + u * kBlock;
    if (i < n4) {
      f4 acc = ZIN ? f4(0.0f) : in[i];
#pragma unroll
      for (int k = 0; k < NB; ++k) acc += ld_stream(bp[k] + i);
      out[i] = acc;
    }
  }
}

// Scalar form: unaligned pointers and the < 4-float tail.
template <int NB, bool ZIN = false, bool GATED = false>
__global__ __launch_bounds__(kBlock) void bucket_sum_scalar_kernel(
    float *__restrict__ out, const float *__restrict__ in, BucketPtrs b,
    size_t n, Gate gate = Gate{}) {
  if constexpr (GATED) {
    if (gate_closed(gate)) return;
  }
  const size_t stride = (size_t)gridDim.x * kBlock;
  for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    float acc = ZIN ? 0.0f : in[i];
#pragma unroll
    for (int k = 0; k < NB; ++k) acc += b.p[k][i];
    out[i] = acc;
  }
}

// Phase-separated form for large shards.  Every byte still moves once, but a
// CU first READS a chunk (master + NB buckets, summed into LDS and registers),
// then WRITES it back, instead of interleaving its loads and stores: on HBM
// the mixed stream loses 10-25 % to read/write interleaving.
// No grid barrier: a launch covers one chunk, and its blocks stay in phase
// because they do identical work and start together (a launch boundary
// re-aligns them).  1 block of 256 threads per CU with the CU's whole LDS
// (160 KiB = 10 tiles of 16 KiB) plus RT register tiles; every access
// non-temporal.  Chunk c covers tiles [c * G * T, (c + 1) * G * T) of kTile
// f4 each; block g takes tiles g, g + G, ...; the first 10 go to LDS, the rest
// to registers.  Only whole tiles: the caller passes n4_tiles, a multiple of
// kTile, and sums any rest with the mixed form.  Shards below 3 chunks are
// cut into C <= 3 balanced chunks (BAL).  The order of the adds per element is
// the bucket order, as in every form.
constexpr int kPhaseLdsF4 = 10240;  // 160 KiB of results per block, 1 block per CU
constexpr int kPhaseU = 4;          // block-strides per tile
constexpr int kPhaseTile = kBlock * kPhaseU;  // f4 per tile (16 KiB)
constexpr int kPhaseLdsTiles = kPhaseLdsF4 / kPhaseTile;
constexpr int kPhaseMinChunks = 3;  // shards below 3 chunks: balanced chunks

template <int NB>
constexpr int phase_reg_tiles() { return NB <= 2 ? 20 : NB <= 4 ? 12 : 4; }

// How a shard of n4_tiles whole tiles is summed: rt < 0 = the mixed form;
// else the phased kernel with rt register tiles, `tiles` tiles per block per
// chunk, `per_launch` chunks per launch, `launches` launches.
struct PhasePlan {
  int rt;
  int tiles;
  int per_launch;
  size_t launches;
  bool balanced;
};

template <int NB>
PhasePlan phase_plan(size_t n4_tiles) {
  const size_t G = (size_t)num_cus();
  const size_t tiles = n4_tiles / kPhaseTile;
  constexpr int rt = phase_reg_tiles<NB>();
  const size_t reg_chunk = G * (kPhaseLdsTiles + rt);
  if (tiles >= reg_chunk * kPhaseMinChunks)  // register-extended chunks, 1 per launch
    return {rt, kPhaseLdsTiles + rt, 1, (tiles + reg_chunk - 1) / reg_chunk, false};
  if (tiles >= G) {  // balanced: C <= 3 chunks of T <= 10 + rt tiles per block
    const size_t chunks = (tiles + reg_chunk - 1) / reg_chunk;
    return {rt, (int)((tiles + G * chunks - 1) / (G * chunks)), 1, chunks, true};
  }
  return {-1, 0, 0, 0, false};
}

// BAL: a balanced chunk of `bal_tiles` (<= kT) tiles per block, one chunk per
// launch.  Otherwise chunks of kT tiles, 1 (register tiles) or 2 per launch,
// all compile-time: the fixed forms measured 18 % slower with the tile count
// and chunks per launch passed at run time: "prod" rows at 200 and 512 MiB
// in profiles/r01b/balance_tune_runtime_tiles.txt.
template <int NB, int RT, bool BAL, bool ZIN = false, bool GATED = false>
__global__ __launch_bounds__(kBlock) void bucket_sum_phased_kernel(
    f4 *__restrict__ out, const f4 *__restrict__ in, BucketPtrs b, size_t n4_tiles,
    size_t chunk0, int bal_tiles, Gate gate = Gate{}) {
  if constexpr (GATED) {
    if (gate_closed(gate)) return;
  }
  constexpr int U = kPhaseU;
  constexpr int kT = kPhaseLdsTiles + RT;
  const int tiles = BAL ? bal_tiles : kT;
  constexpr int per_launch = BAL ? 1 : (RT > 0 ? 1 : 2);
  __shared__ f4 res[kPhaseLdsF4];
  f4 keep[RT > 0 ? RT : 1][U];
  const f4 *bp[NB > 0 ? NB : 1];  // NB = 0: a plain copy out = in (a gather plan's dense runs)
#pragma unroll
  for (int k = 0; k < NB; ++k) bp[k] = reinterpret_cast<const f4 *>(b.p[k]);
  const size_t G = gridDim.x;
  const size_t chunk_f4 = G * (size_t)tiles * kPhaseTile;  // tiles <= kT
  for (int kc = 0; kc < per_launch; ++kc) {
    const size_t lo = (chunk0 + kc) * chunk_f4;
    if (lo >= n4_tiles) return;  // grid-uniform: no block skips a barrier another waits at
    // read phase: sum the chunk's tiles into LDS (t < kPhaseLdsTiles) and registers
#pragma unroll
    for (int t = 0; t < kT; ++t) {
      const size_t tile0 = lo + ((size_t)t * G + blockIdx.x) * kPhaseTile;
      if (t >= tiles || tile0 >= n4_tiles) break;  // block-uniform; later tiles are further out
      const size_t base = tile0 + threadIdx.x;
      f4 acc[U];
      f4 v[NB > 0 ? NB : 1][U];
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u] = ZIN ? f4(0.0f) : ld_stream(in + base + u * kBlock);
#pragma unroll
      for (int k = 0; k < NB; ++k)
#pragma unroll
        for (int u = 0; u < U; ++u) v[k][u] = ld_stream(bp[k] + base + u * kBlock);
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int k = 0; k < NB; ++k) acc[u] += v[k][u];  // bucket order 0..NB-1
        if (t < kPhaseLdsTiles)
          res[t * kPhaseTile + u * kBlock + threadIdx.x] = acc[u];
        else
          keep[t >= kPhaseLdsTiles ? t - kPhaseLdsTiles : 0][u] = acc[u];
      }
    }
    __syncthreads();
    // write phase
#pragma unroll
    for (int t = 0; t < kT; ++t) {
      const size_t tile0 = lo + ((size_t)t * G + blockIdx.x) * kPhaseTile;
      if (t >= tiles || tile0 >= n4_tiles) break;
      const size_t base = tile0 + threadIdx.x;
#pragma unroll
      for (int u = 0; u < U; ++u)
        __builtin_nontemporal_store(t < kPhaseLdsTiles
                                        ? res[t * kPhaseTile + u * kBlock + threadIdx.x]
                                        : keep[t >= kPhaseLdsTiles ? t - kPhaseLdsTiles : 0][u],
                                    out + base + u * kBlock);
    }
    __syncthreads();
  }
}

template <int NB, int RT, bool BAL, bool ZIN = false>
void launch_phased(float *out, const float *in, const BucketPtrs &b, size_t n4_tiles,
                   const PhasePlan &p, hipStream_t s, const Gate *g = nullptr) {
  const size_t G = (size_t)num_cus();
  for (size_t l = 0; l < p.launches; ++l)
    GP_LAUNCH_GATED(NB <= 1, g, (bucket_sum_phased_kernel<NB, RT, BAL, ZIN>),
                    (bucket_sum_phased_kernel<NB, RT, BAL, ZIN, true>), dim3((unsigned)G), dim3(kBlock), s,
                    reinterpret_cast<f4 *>(out), reinterpret_cast<const f4 *>(in), b, n4_tiles,
                    l * (size_t)p.per_launch, p.tiles);
}

// Stream-by-stream ("sweep") form of the phased sum.  Same chunk scheme (LDS
// + register tiles, then a write phase), but the read phase sweeps the
// block's tiles once per stream, in bucket order: pass 0 parks the master's
// (or `in`'s) tiles, pass k adds bucket k-1's tiles into them.  So at any
// moment the chip reads one contiguous region of one stream instead of
// NB + 1 regions at once, with bursts of TG tiles of U block-strides in
// flight per wave.  The per-element order is unchanged, ((in + b0) + b1) +
// ..., so the bits are those of every other form.  ZIN: no `in` stream; pass
// 0 parks 0.0f + b0 (-0 -> +0, as after the memset a row plan's fused init
// replaces).  Shapes (SweepShape; measured per shape in DESIGN.md §5): 96-MiB
// chunks of 32-KiB tiles in bursts of 1 at 2-8 buckets, of 16-KiB tiles in
// bursts of 8 at 1 bucket; 64-MiB chunks in bursts of 4 for the one-stream
// forms (ZIN, the NB = 0 copy) and after the big chunks.  A plan takes whole
// big chunks, then whole 64-MiB chunks (3-8 buckets), then hands the rest to
// the tile-major form.  Whole chunks only (no guards: the waitcnt counts stay
// exact; tests/test_kernel_schedule.py checks the schedule).
template <int NB, bool ZIN>
struct SweepShape {  // the big chunks: register tiles, tiles per burst, block-strides per tile
  // one stream (the zero-input form, the NB = 0 copy): 64-MiB chunks, bursts of 4 16-KiB tiles
  static constexpr bool kOne = ZIN || NB == 0;
  static constexpr int RT = kOne ? 6 : NB == 1 ? 14 : 7;
  static constexpr int TG = kOne ? 4 : NB == 1 ? 8 : 1;
  static constexpr int U = kOne || NB == 1 ? kPhaseU : 8;
  // f4 per block per chunk: the LDS tiles' 160 KiB + the register tiles
  static constexpr size_t kBlockF4 = kPhaseLdsF4 + (size_t)RT * kBlock * U;
};
constexpr int kSweepRT = 6;  // the small (64-MiB) chunks and the zero-input form
constexpr int kSweepTG = 4;
[[maybe_unused]] constexpr int kSweepT = kPhaseLdsTiles + kSweepRT;  // tuning harnesses

// RT register tiles, bursts of TG tiles of U block-strides (4 KiB each)
// (template arguments so the tuning harnesses can instantiate other shapes;
// production uses SweepShape).
template <int NB, int RT = kSweepRT, int TG = kSweepTG, bool ZIN = false, int U = kPhaseU, bool GATED = false>
__global__ __launch_bounds__(kBlock) void bucket_sum_sweep_kernel(
    f4 *__restrict__ out, const f4 *__restrict__ in, BucketPtrs b, size_t n4_tiles,
    size_t chunk, Gate gate = Gate{}) {
  constexpr int kTile = kBlock * U;            // f4 per tile
  constexpr int kLds = kPhaseLdsF4 / kTile;    // tiles parked in LDS
  static_assert(kLds * kTile == kPhaseLdsF4, "whole LDS tiles");
  constexpr int kT = kLds + RT;
  constexpr int S = ZIN ? NB : NB + 1;  // streams read
  static_assert(kT % TG == 0, "whole bursts");
  __shared__ f4 res[kPhaseLdsF4];
  f4 keep[RT][U];
  const f4 *src[S];
#pragma unroll
  for (int k = 0; k < S; ++k)
    src[k] = (!ZIN && k == 0) ? in : reinterpret_cast<const f4 *>(b.p[ZIN ? k : (k > 0 ? k - 1 : 0)]);
  const size_t G = gridDim.x;
  const size_t lo = chunk * G * (size_t)kT * kTile;
  // Never taken (the host launches whole chunks only), but keep it: with this
  // exit the compiler schedules each burst's loads together at 6-8 buckets;
  // without it, short of registers, it regrouped the register tiles' adds
  // into load -> vmcnt(0) -> add chains (117-224 full drains per chunk, 8.3
  // instead of 6.5 ms at 8 buckets; profiles/r01b/sweep_ab.txt).
  // tests/test_kernel_schedule.py checks the schedule on the assembly.
  // GATED: the gate test joins this exit, so its word's load waits on the
  // same first batch of argument loads as the rest of the prologue (a
  // separate test first cost each launch a round trip more, ~1.5 % of a
  // 64-MiB chunk's 21 us).
  bool closed = false;
  if constexpr (GATED) closed = gate_closed(gate);
  if (lo >= n4_tiles || closed) return;
#pragma unroll
  for (int k = 0; k < S; ++k) {
#pragma unroll
    for (int t0 = 0; t0 < kT; t0 += TG) {
      f4 v[TG][U];
#pragma unroll
      for (int j = 0; j < TG; ++j)
#pragma unroll
        for (int u = 0; u < U; ++u)
          v[j][u] = ld_stream(src[k] + lo + ((size_t)(t0 + j) * G + blockIdx.x) * kTile +
                              threadIdx.x + u * kBlock);
#pragma unroll
      for (int j = 0; j < TG; ++j) {
        const int t = t0 + j;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          // each lane owns its slots: no barrier between passes; bucket order 0..NB-1
          const f4 first = ZIN ? f4(0.0f) + v[j][u] : v[j][u];
          if (t < kLds) {
            f4 &r = res[t * kTile + u * kBlock + threadIdx.x];
            r = k == 0 ? first : r + v[j][u];
          } else {
            f4 &r = keep[t >= kLds ? t - kLds : 0][u];
            r = k == 0 ? first : r + v[j][u];
          }
        }
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int t = 0; t < kT; ++t) {
    const size_t base = lo + ((size_t)t * G + blockIdx.x) * kTile + threadIdx.x;
#pragma unroll
    for (int u = 0; u < U; ++u)
      __builtin_nontemporal_store(t < kLds
                                      ? res[t * kTile + u * kBlock + threadIdx.x]
                                      : keep[t >= kLds ? t - kLds : 0][u],
                                  out + base + u * kBlock);
  }
}

// Whole sweep chunks of a shard of n4_tiles f4: `big` chunks of the
// SweepShape (when there are at least kPhaseMinChunks of them), then, at 3-8
// buckets, `small` 64-MiB chunks of what is left (any number after big
// chunks, else at least kPhaseMinChunks); the tile-major plan takes the rest.
struct SweepSplit {
  size_t big = 0, small = 0;
  size_t big_f4 = 0, small_f4 = 0;  // f4 per chunk
  size_t done_f4() const { return big * big_f4 + small * small_f4; }
};

template <int NB, bool ZIN = false>
SweepSplit sweep_split(size_t n4_tiles) {
  using SS = SweepShape<NB, ZIN>;
  const size_t G = (size_t)num_cus();
  SweepSplit sp;
  sp.big_f4 = G * SS::kBlockF4;
  sp.small_f4 = G * (size_t)(kPhaseLdsTiles + kSweepRT) * kPhaseTile;
  sp.big = n4_tiles / sp.big_f4;
  if (sp.big < (size_t)kPhaseMinChunks) sp.big = 0;
  if (!SS::kOne && NB >= 3) {  // at 1-2 buckets the 64-MiB sweep lost to tile-major
    // One big chunk fewer when that lets whole small chunks take more of the
    // rest: a 512-MiB shard is 4 x 96 + 2 x 64 MiB, not 5 x 96 + 32 MiB
    // through the tile-major form.
    if (sp.big > (size_t)kPhaseMinChunks &&
        (n4_tiles - (sp.big - 1) * sp.big_f4) % sp.small_f4 < (n4_tiles - sp.big * sp.big_f4) % sp.small_f4)
      --sp.big;
    sp.small = (n4_tiles - sp.big * sp.big_f4) / sp.small_f4;
    if (sp.big == 0 && sp.small < (size_t)kPhaseMinChunks) sp.small = 0;
  }
  return sp;
}

// Buckets advanced by `off` floats.
template <int NB>
BucketPtrs offset_buckets(const BucketPtrs &b, size_t off) {
  BucketPtrs t = {};
  for (int k = 0; k < NB; ++k) t.p[k] = b.p[k] + off;
  return t;
}

// out[i] = in[i] + b0[i] + ... over i < n: the phase-separated form over the
// whole 16-KiB tiles of a large shard, the mixed dwordx4 form over what is
// left of the 16-B-aligned part, the scalar form over the rest.  ZIN: `in` is
// ignored (may be null) and out[i] = 0.0f + b0[i] + ...  The CU count is read
// once, so the plan and every grid of the call agree.  `g`: every launch gated.
template <int NB, bool ZIN = false>
int launch_bucket_sum_nb(float *out, const float *in, const BucketPtrs &b,
                         size_t n, hipStream_t s, const Gate *g = nullptr) {
  const size_t G = (size_t)num_cus();
  bool vec = aligned16(out) && (ZIN || aligned16(in));
  for (int k = 0; k < NB; ++k) vec = vec && aligned16(b.p[k]);
  size_t done = 0;  // floats summed so far
  if (vec) {
    // whole sweep chunks first, one launch each: big, then small
    using SS = SweepShape<NB, ZIN>;
    const SweepSplit sp = sweep_split<NB, ZIN>(n / 4 / kPhaseTile * kPhaseTile);
    for (size_t c = 0; c < sp.big; ++c)
      GP_LAUNCH_GATED(NB <= 1, g, (bucket_sum_sweep_kernel<NB, SS::RT, SS::TG, ZIN, SS::U>),
                      (bucket_sum_sweep_kernel<NB, SS::RT, SS::TG, ZIN, SS::U, true>), dim3((unsigned)G),
                      dim3(kBlock), s, reinterpret_cast<f4 *>(out), reinterpret_cast<const f4 *>(in), b,
                      n / 4, c);
    done = sp.big * sp.big_f4 * 4;
    if constexpr (!SS::kOne) {
      const BucketPtrs bo = offset_buckets<NB>(b, done);
      for (size_t c = 0; c < sp.small; ++c)
        GP_LAUNCH_GATED(NB <= 1, g, (bucket_sum_sweep_kernel<NB, kSweepRT, kSweepTG, ZIN>),
                        (bucket_sum_sweep_kernel<NB, kSweepRT, kSweepTG, ZIN, kPhaseU, true>), dim3((unsigned)G),
                        dim3(kBlock), s, reinterpret_cast<f4 *>(out + done),
                        reinterpret_cast<const f4 *>(ZIN ? nullptr : in + done), bo, (n - done) / 4, c);
      done += sp.small * sp.small_f4 * 4;
    }
    // the rest (all of it below 3 sweep chunks): the tile-major phased form
    const size_t n4_tiles = (n - done) / 4 / kPhaseTile * kPhaseTile;
    const PhasePlan p = phase_plan<NB>(n4_tiles);
    if (p.rt >= 0) {
      const BucketPtrs bo = offset_buckets<NB>(b, done);
      const float *ip = ZIN ? nullptr : in + done;
      if (p.balanced)
        launch_phased<NB, phase_reg_tiles<NB>(), true, ZIN>(out + done, ip, bo, n4_tiles, p, s, g);
      else
        launch_phased<NB, phase_reg_tiles<NB>(), false, ZIN>(out + done, ip, bo, n4_tiles, p, s, g);
      done += n4_tiles * 4;
    }
  }
  const float *in_at = ZIN ? nullptr : in + done;
  if (vec && n - done >= 4) {
    // 4 block-strides per thread at 2 blocks per CU: (NB + 1) * 4 dwordx4 loads
    // in flight per lane.  Measured on MI355X at 8 x 4 GiB buckets: +2-3 % over
    // 1 stride at 8 blocks/CU (profiles/r01/bucket_tune_sweep*.txt).
    constexpr int U = 4;
    constexpr int kPerCU = NB <= 2 ? 4 : 2;
    const size_t n4 = (n - done) / 4;
    const size_t tiles = (n4 + (size_t)kBlock * U - 1) / ((size_t)kBlock * U);
    const size_t cap = G * kPerCU;
    const size_t grid = tiles < cap ? tiles : cap;
    GP_LAUNCH_GATED(NB <= 1, g, (bucket_sum_vec_kernel<NB, U, ZIN>), (bucket_sum_vec_kernel<NB, U, ZIN, true>),
                    dim3((unsigned)grid), dim3(kBlock), s, reinterpret_cast<f4 *>(out + done),
                    reinterpret_cast<const f4 *>(in_at), offset_buckets<NB>(b, done), n4);
    done += n4 * 4;
    in_at = ZIN ? nullptr : in + done;
  }
  if (done < n) {
    const size_t rem = n - done;
    size_t grid = (rem + kBlock - 1) / kBlock;
    if (grid > G * kBlocksPerCU) grid = G * kBlocksPerCU;
    GP_LAUNCH_GATED(NB <= 1, g, (bucket_sum_scalar_kernel<NB, ZIN>), (bucket_sum_scalar_kernel<NB, ZIN, true>),
                    dim3((unsigned)grid), dim3(kBlock), s, out + done, in_at, offset_buckets<NB>(b, done), rem);
  }
  GP_HIP_TRY(hipGetLastError());
  return GP_OK;
}

// Launch plan of one pass of NB buckets over n 16-B-aligned floats, as
// launch_bucket_sum_nb issues it (bench.py prices the dominant kernel per
// launch with it).
struct SumLaunches {
  size_t sweep = 0, sweep_small = 0, phased = 0, other = 0;
  int reg_tiles = -1;  // the dominant phased form's register tiles
  int phased_reg_tiles = -1;
};

template <int NB, bool ZIN = false>
SumLaunches sum_launches(size_t n) {
  constexpr int RT = SweepShape<NB, ZIN>::RT;
  SumLaunches l;
  const SweepSplit sp = sweep_split<NB, ZIN>(n / 4 / kPhaseTile * kPhaseTile);
  l.sweep = sp.big;
  l.sweep_small = sp.small;
  size_t done = sp.done_f4() * 4;
  const size_t n4_tiles = (n - done) / 4 / kPhaseTile * kPhaseTile;
  const PhasePlan p = phase_plan<NB>(n4_tiles);
  if (p.rt >= 0) {
    l.phased = p.launches;
    l.phased_reg_tiles = p.rt;
    done += n4_tiles * 4;
  }
  l.reg_tiles = sp.big ? RT : sp.small ? kSweepRT : p.rt;
  if (n - done >= 4) {
    l.other++;
    done += (n - done) / 4 * 4;
  }
  if (done < n) l.other++;
  return l;
}

template <int NB>
void bucket_sum_plan_nb(size_t n, int *launches, int *reg_tiles, int *sweep_launches) {
  const SumLaunches l = sum_launches<NB>(n);
  *sweep_launches = (int)(l.sweep + l.sweep_small);
  *reg_tiles = l.reg_tiles;
  *launches = (int)(l.sweep + l.sweep_small + l.phased);
}

template <int NB>
void sum_plan_nb(size_t n, gp_sum_plan *out) {
  const SumLaunches l = sum_launches<NB>(n);
  out->sweep_launches = (int)l.sweep;
  out->sweep_reg_tiles = l.sweep ? SweepShape<NB, false>::RT : -1;
  out->sweep_burst_tiles = l.sweep ? SweepShape<NB, false>::TG : -1;
  out->sweep_tile_kib = l.sweep ? SweepShape<NB, false>::U * 4 : -1;
  out->small_sweep_launches = (int)l.sweep_small;
  out->small_sweep_burst_tiles = l.sweep_small ? kSweepTG : -1;
  out->phased_launches = (int)l.phased;
  out->phased_reg_tiles = l.phased_reg_tiles;
  out->other_launches = (int)l.other;
}

inline int launch_bucket_sum(float *out, const float *in, const float *const *bk,
                      int nb, size_t n, hipStream_t s) {
  BucketPtrs b = {};
  for (int k = 0; k < nb; ++k) b.p[k] = bk[k];
  switch (nb) {
    case 1: return launch_bucket_sum_nb<1>(out, in, b, n, s);
    case 2: return launch_bucket_sum_nb<2>(out, in, b, n, s);
    case 3: return launch_bucket_sum_nb<3>(out, in, b, n, s);
    case 4: return launch_bucket_sum_nb<4>(out, in, b, n, s);
    case 5: return launch_bucket_sum_nb<5>(out, in, b, n, s);
    case 6: return launch_bucket_sum_nb<6>(out, in, b, n, s);
    case 7: return launch_bucket_sum_nb<7>(out, in, b, n, s);
    case 8: return launch_bucket_sum_nb<8>(out, in, b, n, s);
    default: return set_error(GP_ERR_INVALID, "bucket count out of range");
  }
}

// ---------------------------------------------------------------------------
// Row-indexed ops over a DoubleIndex.
// ---------------------------------------------------------------------------

enum RowOp : int {
  kAddFrom = 0,     // y[id1] += x[id0], guard on the x index
  kAssignTo = 1,    // y[id0]  = x[id1], guard on the y index
  kAssignFrom = 2,  // y[id1]  = x[id0], guard on the x index
  kInitFrom = 3,    // y[id1]  = 0.0f + x[id0] (0.0f where the x index is guarded out)
};

template <int OP>
__device__ __forceinline__ void row_endpoints(const gp_double_index &ix,
                                              uint64_t off0, uint64_t off1,
                                              uint64_t &from, uint64_t &to) {
  if (OP == kAssignTo) {
    from = ix.id1 + off1;
    to = ix.id0 + off0;
  } else {
    from = ix.id0 + off0;
    to = ix.id1 + off1;
  }
}

// Where the cache side of a row op lives.  kFlat: one buffer (x or y as
// passed).  kSegX / kSegY: the cache rows (`from` of a gather / `to` of a
// scatter-add) are split over the buffers of a gp_row_segments table, passed
// by value as a kernel argument.
enum SegMode : int { kFlat = 0, kSegX = 1, kSegY = 2 };

template <int SEG>
struct SegArg {};
template <>
struct SegArg<kSegX> {
  gp_row_segments t;
};
template <>
struct SegArg<kSegY> {
  gp_row_segments t;
};

// Segment i holding cache row `row` (first_row ascending, first_row[0] == 0).
__device__ __forceinline__ float *seg_row(const gp_row_segments &t, uint64_t row,
                                          size_t row_size) {
  uint32_t s = 0;
  for (uint32_t i = 1; i < t.count; ++i) s += (t.first_row[i] <= row) ? 1u : 0u;
  return t.base[s] + (row - t.first_row[s]) * row_size;
}

// Cache policy of row_op_kernel / row_op_seg_kernel per stream (DESIGN.md
// §5): the op buffer x of a scatter-add / init is read once per call, with
// non-temporal loads; the oplog side stays plain; the gather (Read) uses
// non-temporal loads of the cache rows AND stores into the op buffer.
// row_wave_kernel (the sorted residuals, the gather, the op-order init) has
// its own policy: non-temporal on every access.
template <int OP, typename T>
__device__ __forceinline__ T ld_src(const T *p) {
  if constexpr (OP == kAddFrom || OP == kInitFrom || OP == kAssignTo)
    return __builtin_nontemporal_load(p);
  else
    return *p;
}

template <int OP, typename T>
__device__ __forceinline__ void st_copy(T *p, T v) {
  if constexpr (OP == kAssignTo)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

// T = f4 (VEC 4) or float (VEC 1).  A group of LPR consecutive lanes owns a
// row; each group handles RPG rows per iteration, all their loads issued
// before the first store.  `vw` = row_size / VEC (vectors per row).
template <typename T, int VEC, int OP, int LPR, int RPG, bool GATED = false>
__global__ __launch_bounds__(kBlock) void row_op_kernel(
    float *__restrict__ y, const float *__restrict__ x,
    const gp_double_index *__restrict__ index, size_t num_rows, uint64_t off0,
    uint64_t off1, size_t row_size, size_t vw, size_t limit, Gate gate = Gate{}) {
  if constexpr (GATED) GP_ROW_GATE(gate, index, num_rows, off0, off1);
  constexpr int kGroups = kBlock / LPR;
  const int lane = threadIdx.x % LPR;
  const size_t group = (size_t)blockIdx.x * kGroups + threadIdx.x / LPR;
  const size_t gstride = (size_t)gridDim.x * kGroups * RPG;
  T *yv = reinterpret_cast<T *>(y);
  const T *xv = reinterpret_cast<const T *>(x);

  for (size_t r0 = group * RPG; r0 < num_rows; r0 += gstride) {
    uint64_t from[RPG], to[RPG];
    bool live[RPG], whole[RPG];
#pragma unroll
    for (int k = 0; k < RPG; ++k) {
      const size_t r = r0 + k;
      live[k] = r < num_rows;
      from[k] = to[k] = 0;
      whole[k] = false;
      if (live[k]) {
        const gp_double_index ix = index[r];
        row_endpoints<OP>(ix, off0, off1, from[k], to[k]);
        const uint64_t guarded = (OP == kAssignTo) ? to[k] : from[k];
        whole[k] = (guarded + 1) * row_size <= limit;
      }
    }
    bool all_whole = true;
#pragma unroll
    for (int k = 0; k < RPG; ++k) all_whole = all_whole && (whole[k] || !live[k]);

    if (all_whole) {
      for (size_t j = lane; j < vw; j += LPR) {
        T xs[RPG], ys[RPG];
#pragma unroll
        for (int k = 0; k < RPG; ++k)
          if (live[k]) xs[k] = ld_src<OP>(xv + from[k] * vw + j);
        if (OP == kAddFrom) {
#pragma unroll
          for (int k = 0; k < RPG; ++k)
            if (live[k]) ys[k] = yv[to[k] * vw + j];
        }
#pragma unroll
        for (int k = 0; k < RPG; ++k) {
          if (live[k]) {
            if (OP == kAddFrom)
              yv[to[k] * vw + j] = ys[k] + xs[k];
            else if (OP == kInitFrom)
              yv[to[k] * vw + j] = T(0.0f) + xs[k];  // == zerofy then +=, -0 -> +0 included
            else
              st_copy<OP>(yv + to[k] * vw + j, xs[k]);
          }
        }
      }
    } else {
      // Rows straddling num_vals_limit: element-wise guard, scalar accesses
      // (nothing past the limit is touched, as in the reference).
#pragma unroll 1
      for (int k = 0; k < RPG; ++k) {
        if (!live[k]) continue;
        const uint64_t guarded = (OP == kAssignTo) ? to[k] : from[k];
        for (size_t e = lane; e < row_size; e += LPR) {
          if (guarded * row_size + e < limit) {
            const float xv1 = x[from[k] * row_size + e];
            if (OP == kAddFrom)
              y[to[k] * row_size + e] += xv1;
            else if (OP == kInitFrom)
              y[to[k] * row_size + e] = 0.0f + xv1;
            else
              y[to[k] * row_size + e] = xv1;
          } else if (OP == kInitFrom) {
            y[to[k] * row_size + e] = 0.0f;  // the zerofied value the add never touched
          }
        }
      }
    }
  }
}

// Segmented form (kSegX: gather from the segmented cache; kSegY: scatter-add
// into it): the same lane/row mapping, with each cache-side row resolved to a
// pointer through the segment table once per row.  A separate kernel so the
// flat kernels above keep their register budget.
template <typename T, int VEC, int OP, int LPR, int RPG, int SEG>
__global__ __launch_bounds__(kBlock) void row_op_seg_kernel(
    float *__restrict__ y, const float *__restrict__ x,
    const gp_double_index *__restrict__ index, size_t num_rows, uint64_t off0,
    uint64_t off1, size_t row_size, size_t vw, size_t limit, const SegArg<SEG> seg) {
  static_assert(SEG == kSegX || SEG == kSegY, "segmented side");
  constexpr int kGroups = kBlock / LPR;
  const int lane = threadIdx.x % LPR;
  const size_t group = (size_t)blockIdx.x * kGroups + threadIdx.x / LPR;
  const size_t gstride = (size_t)gridDim.x * kGroups * RPG;

  for (size_t r0 = group * RPG; r0 < num_rows; r0 += gstride) {
    uint64_t guarded[RPG];
    const float *xr[RPG];
    float *yr[RPG];
    bool live[RPG], whole[RPG];
#pragma unroll
    for (int k = 0; k < RPG; ++k) {
      const size_t r = r0 + k;
      live[k] = r < num_rows;
      guarded[k] = 0;
      xr[k] = x;
      yr[k] = y;
      whole[k] = false;
      if (live[k]) {
        const gp_double_index ix = index[r];
        uint64_t from, to;
        row_endpoints<OP>(ix, off0, off1, from, to);
        guarded[k] = (OP == kAssignTo) ? to : from;
        whole[k] = (guarded[k] + 1) * row_size <= limit;
        xr[k] = SEG == kSegX ? seg_row(seg.t, from, row_size) : x + from * row_size;
        yr[k] = SEG == kSegY ? seg_row(seg.t, to, row_size) : y + to * row_size;
      }
    }
    bool all_whole = true;
#pragma unroll
    for (int k = 0; k < RPG; ++k) all_whole = all_whole && (whole[k] || !live[k]);

    if (all_whole) {
      for (size_t j = lane; j < vw; j += LPR) {
        T xs[RPG], ys[RPG];
#pragma unroll
        for (int k = 0; k < RPG; ++k)
          if (live[k]) xs[k] = ld_src<OP>(reinterpret_cast<const T *>(xr[k]) + j);
        if (OP == kAddFrom) {
#pragma unroll
          for (int k = 0; k < RPG; ++k)
            if (live[k]) ys[k] = reinterpret_cast<const T *>(yr[k])[j];
        }
#pragma unroll
        for (int k = 0; k < RPG; ++k)
          if (live[k])
            st_copy<OP>(reinterpret_cast<T *>(yr[k]) + j, OP == kAddFrom ? ys[k] + xs[k] : xs[k]);
      }
    } else {
#pragma unroll 1
      for (int k = 0; k < RPG; ++k) {
        if (!live[k]) continue;
        for (size_t e = lane; e < row_size; e += LPR)
          if (guarded[k] * row_size + e < limit) {
            if (OP == kAddFrom)
              yr[k][e] += xr[k][e];
            else
              yr[k][e] = xr[k][e];
          }
      }
    }
  }
}

__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
  const int lo = __shfl((int)(uint32_t)v, src, 64);
  const int hi = __shfl((int)(uint32_t)(v >> 32), src, 64);
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

// Wave-level index map for rows of up to 128 floats (LPR <= 32 lanes per
// row, 2 or more rows per wave instruction).  Lane l of a wave loads entry
// t + l of the wave's 64-row tile -- one coalesced 1-KiB read -- and resolves
// it to a source pointer (flat cache, or the segmented cache's buffer), a
// destination pointer and the row's num_vals_limit guard; the row groups take
// theirs by __shfl.  The next tile's entries load while this tile's rows move,
// so no row load waits on an index load.  Used for the gather (flat and
// segmented), the fused init, and the scatter-add of destination-sorted rows
// (a row plan's residual, a device-binned residual); in op order the
// scatter-add keeps row_op_kernel.  Every access non-temporal.
// MAP 0 (production): wave w takes tiles w, w + waves, ... (grid-stride).
// MAP 2 (tuning harnesses only): the blocks of one XCD -- dealt round-robin,
// so blocks b and b + 8 share one (MI355X_MICROARCH.md, workgroup dispatch)
// -- take one contiguous eighth of the tiles, grid-stride inside it; needs a
// multiple of 8 blocks.  It tied or lost on a random index (probe 8,
// profiles/r03/tune/r3_tilemap_tune.txt).
template <typename T, int OP, int LPR, int RPG, int SEG, int MAP = 0, bool GATED = false>
__global__ __launch_bounds__(kBlock) void row_wave_kernel(
    float *__restrict__ y, const float *__restrict__ x,
    const gp_double_index *__restrict__ index, size_t num_rows, uint64_t off0,
    uint64_t off1, size_t row_size, size_t vw, size_t limit, const SegArg<SEG> seg, Gate gate = Gate{}) {
  const uint64_t *inv = nullptr;  // GATED: the inverse map walked instead of `index`
  if constexpr (GATED) {
    if (gate.mode == kGateSelect && gate_changed(gate)) {
      index = gate.alt;
      num_rows = gate.alt_rows;
      off0 = gate.alt_off0;
      off1 = gate.alt_off1;
    } else if (gate_closed(gate)) {
      return;
    } else {
      inv = gate.inv;
    }
  }
  static_assert((OP == kAssignTo && (SEG == kFlat || SEG == kSegX)) ||
                    ((OP == kAddFrom || OP == kInitFrom) && SEG == kFlat),
                "gather (flat / segmented source) or flat scatter-add / init");
  // Row pointers travel through __shfl as integers; accessed as global-address-
  // space pointers so the loads and stores stay global_* (a generic pointer
  // would make them flat_*, measured 2x slower here).  The gather's cache
  // policy (ld_src / st_copy): non-temporal both ways.
  typedef __attribute__((address_space(1))) T GT;
  constexpr int kG = 64 / LPR;            // row groups per wave
  constexpr int kRowsPerGroup = 64 / kG;  // rows of a 64-row tile per group
  constexpr int kRPG = RPG < kRowsPerGroup ? RPG : kRowsPerGroup;
  const int wl = threadIdx.x & 63, lane = wl % LPR, gw = wl / LPR;
  const size_t wave = ((size_t)blockIdx.x * kBlock + threadIdx.x) / 64;
  const size_t wstride = (size_t)gridDim.x * (kBlock / 64) * 64;
  // MAP 2: this XCD's region of tiles [r0, r1) (rows), walked from lw by lstride
  size_t r1 = num_rows, lstride = wstride;
  size_t t = wave * 64;
  if constexpr (MAP == 2) {
    const size_t tiles = (num_rows + 63) / 64, region = (tiles + 7) / 8 * 64;
    const size_t xcd = blockIdx.x % 8, per = gridDim.x / 8;
    const size_t lw = (blockIdx.x / 8) * (kBlock / 64) + threadIdx.x / 64;
    lstride = per * (kBlock / 64) * 64;
    const size_t r0 = xcd * region;
    r1 = r0 + region < num_rows ? r0 + region : num_rows;
    t = r0 + lw * 64;
  }
  if (t >= r1) return;  // wave-uniform: every lane of a wave reaches each __shfl

  // this lane's row of the current tile: source / destination row pointers,
  // and whether the row is clear of num_vals_limit (guarded on the
  // destination row for the gather, as in the reference's assign-to, and on
  // the source row for the scatter ops)
  uint64_t msrc = 0, mdst = 0;
  int mwhole = 0;
  auto resolve = [&](const gp_double_index &ix, bool live) {
    msrc = mdst = 0;
    mwhole = 0;
    if (!live) return;
    uint64_t from, to;
    row_endpoints<OP>(ix, off0, off1, from, to);
    const float *src;
    if constexpr (SEG == kSegX)
      src = seg_row(seg.t, from, row_size);
    else
      src = x + from * row_size;
    msrc = reinterpret_cast<uint64_t>(src);
    mdst = reinterpret_cast<uint64_t>(y + to * row_size);
    mwhole = ((OP == kAssignTo ? to : from) + 1) * row_size <= limit;
  };
  // entry r of the rows walked: the index's, or (inverse map) destination row
  // r and its source, offsets applied; a row the map does not list is dead
  auto load = [&](size_t r, bool &live) {
    if constexpr (GATED) {
      if (inv) {
        const uint64_t v = inv[r];
        live = live && v != ~0ull;
        return gp_double_index{v & 0xffffffffu, r};
      }
    }
    return index[r];
  };
  {
    bool live = t + wl < num_rows;
    gp_double_index ix = {0, 0};
    if (live) ix = load(t + wl, live);
    resolve(ix, live);
  }
  for (; t < r1; t += lstride) {
    const size_t nr = t + lstride + wl;  // next tile's entry, in flight meanwhile
    bool nlive = MAP == 2 ? t + lstride < r1 && nr < num_rows : nr < num_rows;
    gp_double_index nix = {0, 0};
    if (nlive) nix = load(nr, nlive);
    const size_t rows_here = num_rows - t < 64 ? num_rows - t : 64;
    for (int i0 = 0; i0 < kRowsPerGroup; i0 += kRPG) {
      uint64_t sp[kRPG], dp[kRPG];
      bool live[kRPG];
      bool all_whole = true;
#pragma unroll
      for (int k = 0; k < kRPG; ++k) {
        const int rt = gw + kG * (i0 + k);
        live[k] = (size_t)rt < rows_here;
        sp[k] = shfl64(msrc, rt);
        dp[k] = shfl64(mdst, rt);
        if constexpr (GATED) live[k] = live[k] && dp[k] != 0;  // (an inverse map's unlisted row)
        all_whole = all_whole && (!live[k] || __shfl(mwhole, rt, 64));
      }
      if (all_whole) {  // group-uniform
        for (size_t j = lane; j < vw; j += LPR) {
          T xs[kRPG], ys[kRPG];
#pragma unroll
          for (int k = 0; k < kRPG; ++k)
            if (live[k]) xs[k] = __builtin_nontemporal_load(reinterpret_cast<const GT *>(sp[k]) + j);
          if (OP == kAddFrom) {
#pragma unroll
            for (int k = 0; k < kRPG; ++k)
              if (live[k]) ys[k] = __builtin_nontemporal_load(reinterpret_cast<const GT *>(dp[k]) + j);
          }
#pragma unroll
          for (int k = 0; k < kRPG; ++k) {
            if (!live[k]) continue;
            GT *d = reinterpret_cast<GT *>(dp[k]) + j;
            if (OP == kAddFrom)
              __builtin_nontemporal_store(ys[k] + xs[k], d);
            else if (OP == kInitFrom)
              __builtin_nontemporal_store(T(0.0f) + xs[k], d);  // == zerofy then +=, -0 -> +0
            else
              __builtin_nontemporal_store(xs[k], d);
          }
        }
      } else {
        // rows straddling num_vals_limit: element-wise guard, scalar accesses
        // (k unrolled: a runtime k would index the sp / dp register arrays,
        // which costs the whole kernel registers)
#pragma unroll
        for (int k = 0; k < kRPG; ++k) {
          if (!live[k]) continue;
          const float *xr = reinterpret_cast<const float *>(sp[k]);
          float *yr = reinterpret_cast<float *>(dp[k]);
          // the guarded row: destination of a gather, (flat) source otherwise
          const uint64_t g = OP == kAssignTo ? (uint64_t)(yr - y) / row_size
                                             : (uint64_t)(xr - x) / row_size;
          for (size_t e = lane; e < row_size; e += LPR) {
            if (g * row_size + e < limit) {
              if (OP == kAddFrom)
                yr[e] += xr[e];
              else if (OP == kInitFrom)
                yr[e] = 0.0f + xr[e];
              else
                yr[e] = xr[e];
            } else if (OP == kInitFrom) {
              yr[e] = 0.0f;  // the zerofied value the add never touched
            }
          }
        }
      }
    }
    resolve(nix, nlive);
  }
}

// Blocks of `kernel` resident on one CU at kBlock threads (its register and
// LDS use), cached per instantiation through `cache`.
inline int resident_blocks(const void *kernel, std::atomic<int> &cache) {
  int occ = cache.load(std::memory_order_relaxed);
  if (occ > 0) return occ;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel, kBlock, 0) != hipSuccess || occ <= 0)
    occ = 2;
  cache.store(occ, std::memory_order_relaxed);
  return occ;
}

// Which row kernel moves a call's rows (the index map, the grid).  `sorted`:
// the rows come from a row plan, in ascending destination order.
template <typename T, int VEC, int OP, int SEG, int LPR>
void launch_row_op_lpr(float *y, const float *x, const gp_double_index *idx,
                       size_t n, uint64_t off0, uint64_t off1, size_t row_size,
                       size_t limit, const SegArg<SEG> &seg, bool sorted, hipStream_t s,
                       const Gate *g) {
  constexpr bool kWaveShape = VEC == 4 && LPR <= 32;
  // the unplanned calls' steady state gates its flat launches
  constexpr bool kGatable = SEG == kFlat;
  constexpr bool kWaveGather = OP == kAssignTo && (SEG == kFlat || SEG == kSegX);
  constexpr bool kWaveScatter = (OP == kAddFrom || OP == kInitFrom) && SEG == kFlat;
  if constexpr (kWaveShape && (kWaveGather || kWaveScatter)) {
    // Wave-level index map (row_wave_kernel): the gather of rows up to 128
    // floats, the fused init always, the scatter-add when its rows are sorted
    // by destination.  Rows in flight per group: 8 at 32 lanes per row (16
    // spill past 256 VGPRs), 16 at 16 lanes.
    constexpr int RPG = LPR == 32 ? 8 : 16;
    if (kWaveGather || OP == kInitFrom || sorted) {
      auto *kern = &row_wave_kernel<T, OP, LPR, RPG, SEG>;
      size_t grid = (n + kBlock - 1) / kBlock;  // one 64-row tile per wave
      // One resident round of blocks: every block resident from the start,
      // none waiting for a slot.
      static std::atomic<int> occ{0};
      const size_t cap = (size_t)num_cus() * resident_blocks(reinterpret_cast<const void *>(kern), occ);
      if (grid > cap) grid = cap;
      GP_LAUNCH_GATED(kGatable, g, kern, (row_wave_kernel<T, OP, LPR, RPG, SEG, 0, true>), dim3((unsigned)grid),
                      dim3(kBlock), s, y, x, idx, n, off0, off1, row_size, row_size / VEC, limit, seg);
      return;
    }
  }
  // Keep ~8 independent 16-B loads per lane in flight.
  constexpr int RPG = (OP == kAddFrom) ? 4 : 8;
  constexpr int kGroups = kBlock / LPR;
  const size_t groups = (n + RPG - 1) / RPG;
  size_t grid = (groups + kGroups - 1) / kGroups;
  // The op-order scatter-add of RowData-sized rows at 2 blocks per CU (4 for
  // the segmented form): fewer rows in flight, a narrower window of the
  // read-modify-write side's addresses.
  constexpr bool kRowAdd = OP == kAddFrom && VEC == 4 && LPR == 32;
  const size_t cap = (kRowAdd && SEG == kFlat)   ? (size_t)num_cus() * 2
                     : (kRowAdd && SEG == kSegY) ? (size_t)num_cus() * 4
                                                 : grid_cap();
  if (grid > cap) grid = cap;
  if constexpr (SEG == kFlat)
    GP_LAUNCH_GATED(kGatable, g, (row_op_kernel<T, VEC, OP, LPR, RPG>), (row_op_kernel<T, VEC, OP, LPR, RPG, true>),
                    dim3((unsigned)grid), dim3(kBlock), s, y, x, idx, n, off0, off1, row_size,
                    row_size / VEC, limit);
  else  // (never gated)
    hipLaunchKernelGGL((row_op_seg_kernel<T, VEC, OP, LPR, RPG, SEG>), dim3((unsigned)grid),
                       dim3(kBlock), 0, s, y, x, idx, n, off0, off1, row_size,
                       row_size / VEC, limit, seg);
}

template <typename T, int VEC, int OP, int SEG>
void launch_row_op_t(float *y, const float *x, const gp_double_index *idx,
                     size_t n, uint64_t off0, uint64_t off1, size_t row_size,
                     size_t limit, const SegArg<SEG> &seg, bool sorted, hipStream_t s,
                     const Gate *g = nullptr) {
  const size_t vw = row_size / VEC;
  // Lanes per row: the smallest power of two covering the row, capped at a
  // wave; short rows (64 / 128 floats) pack 4 / 2 rows into one wave.
#define GP_LPR(L) launch_row_op_lpr<T, VEC, OP, SEG, L>(y, x, idx, n, off0, off1, row_size, limit, seg, sorted, s, g)
  if (vw <= 1)
    GP_LPR(1);
  else if (vw <= 2)
    GP_LPR(2);
  else if (vw <= 4)
    GP_LPR(4);
  else if (vw <= 8)
    GP_LPR(8);
  else if (vw <= 16)
    GP_LPR(16);
  else if (vw <= 32)
    GP_LPR(32);
  else
    GP_LPR(64);
#undef GP_LPR
}

template <int OP>
int launch_row_op(float *y, const float *x, const gp_double_index *idx,
                  size_t n, gp_double_index off, size_t row_size, size_t limit,
                  hipStream_t s, bool sorted = false, const Gate *g = nullptr) {
  if (n == 0) return GP_OK;
  if (!y || !x || !idx) return set_error(GP_ERR_INVALID, "null pointer");
  if (row_size == 0) return set_error(GP_ERR_INVALID, "row_size == 0");
  const SegArg<kFlat> flat{};
  if (row_size % 4 == 0 && aligned16(y) && aligned16(x))
    launch_row_op_t<f4, 4, OP, kFlat>(y, x, idx, n, off.id0, off.id1, row_size, limit, flat, sorted,
                                      s, g);
  else
    launch_row_op_t<float, 1, OP, kFlat>(y, x, idx, n, off.id0, off.id1, row_size, limit, flat,
                                         sorted, s, g);
  GP_HIP_TRY(hipGetLastError());
  return GP_OK;
}

inline int check_segments(const gp_row_segments *t, size_t row_size, bool *aligned) {
  if (!t) return set_error(GP_ERR_INVALID, "null segment table");
  if (t->count < 1 || t->count > GP_MAX_SEGMENTS)
    return set_error(GP_ERR_INVALID, "segment count out of range");
  if (t->first_row[0] != 0) return set_error(GP_ERR_INVALID, "first_row[0] != 0");
  *aligned = row_size % 4 == 0;
  for (uint32_t i = 0; i < t->count; ++i) {
    if (!t->base[i]) return set_error(GP_ERR_INVALID, "null segment base");
    if (i && t->first_row[i] <= t->first_row[i - 1])
      return set_error(GP_ERR_INVALID, "segment first_row not ascending");
    *aligned = *aligned && aligned16(t->base[i]);
  }
  return GP_OK;
}

// Segmented cache side: OP kAssignTo reads it (kSegX), kAddFrom writes it (kSegY).
template <int OP, int SEG>
int launch_row_op_seg(float *flat_ptr, const gp_row_segments *t,
                      const gp_double_index *idx, size_t n, gp_double_index off,
                      size_t row_size, size_t limit, hipStream_t s) {
  if (n == 0) return GP_OK;
  if (!flat_ptr || !idx) return set_error(GP_ERR_INVALID, "null pointer");
  if (row_size == 0) return set_error(GP_ERR_INVALID, "row_size == 0");
  bool vec = false;
  const int rc = check_segments(t, row_size, &vec);
  if (rc != GP_OK) return rc;
  vec = vec && aligned16(flat_ptr);
  SegArg<SEG> seg;
  seg.t = *t;
  // the flat side is y for a gather (kSegX) and x for a scatter-add (kSegY)
  float *y = SEG == kSegX ? flat_ptr : nullptr;
  const float *x = SEG == kSegY ? flat_ptr : nullptr;
  if (vec)
    launch_row_op_t<f4, 4, OP, SEG>(y, x, idx, n, off.id0, off.id1, row_size, limit, seg, false, s);
  else
    launch_row_op_t<float, 1, OP, SEG>(y, x, idx, n, off.id0, off.id1, row_size, limit, seg, false,
                                       s);
  GP_HIP_TRY(hipGetLastError());
  return GP_OK;
}

// Dense id0 / id1 runs (row plans, gp_reduce.hip; the unplanned calls' scan,
// gp_unplanned.hip) of at least this many bytes go to the sum kernels above.
// A dense run launches 1-3 kernels; below 4 MiB (the phased form's smallest
// shard) the row kernel moves it without the launches.
constexpr size_t kDenseRunBytes = 4u << 20;

}  // namespace

#endif  // GP_KERNELS_HPP_
