// gp_reduce.hip — gfx950 (MI355X / CDNA4) kernels of the GeePS gradient-update
// reduction path, behind the C-ABI declared in include/gp_reduce.h.
//
// Two kernel families, both HBM-bandwidth bound (elementwise fp32 add; no
// MFMA — there is no contraction here):
//
//  * bucket_sum_*_kernel — the server's N-way sum of client delta buckets into
//    the master shard (reference: TabletStorage::apply_updates,
//    src/server/tablet-server.cpp:119-134, applied once per client message).
//    The reference makes N sequential passes over the shard (3 streams x 4 B
//    per element per client); here one pass reads master + N buckets once and
//    writes master once, summing in bucket order so every element is
//    bit-identical to the sequential form.  Shards of 4 MiB and up use the
//    phase-separated forms (reads of a chunk summed into LDS and registers,
//    then written): whole 96-MiB / 64-MiB chunks by the stream-by-stream
//    sweep, the rest tile-major; smaller ones and leftovers the mixed dwordx4
//    form, then a scalar tail.  NB = 0 is a plain copy and the zero-input
//    (ZIN) form computes 0.0f + b0: the row plans' dense runs (below).
//
//  * row_op_kernel / row_wave_kernel — the row-indexed scatter-add / gather /
//    scatter-assign over a DoubleIndex (reference: src/common/row-op-util.cu:
//    39-142).  The reference launches one thread per ELEMENT with a 64-bit
//    div/mod and a 16-B index load per element; here a group of LPR lanes
//    owns a row, the row's index is loaded once per row (or once per wave and
//    shared by __shfl), and each lane moves 16 B per access (dwordx4), RPG
//    rows per group in flight.
//
//  * row plans — a fixed DoubleIndex compiled once (libgeeps' ops): dense
//    id0/id1 runs go to the bucket-sum kernels above (1 bucket for the
//    scatter-add, ZIN for the fused init, NB = 0 for the gather), the other
//    rows to the row kernels in destination order.
//
//  * the unplanned calls' device planning ("Device-built plans" below): the
//    reference binding's calls pass a device index every call; large calls
//    scan it on the device, build an inverse map / sorted residual / ranges
//    plan once, and from the second call on check the index on the device and
//    run the cached plan with no host round trip (the plan cache, its gated
//    launches and stream-ordered retirement).
//
//  * the C-ABI entry points (the `extern "C"` block at the end).
//
// The library's other translation units: gp_sort.hip (hipCUB radix sort),
// gp_runtime.hip (runtime helpers and IPC, no kernels), gp_host.cpp (the host
// row ops).  Wave64 throughout: 256-thread workgroups = 4 waves, one per SIMD.

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

// gp_sort.hip (hipCUB's radix sort, in its own translation unit): sort n
// (key, value) pairs by the low end_bit bits of the key, stream-ordered, on
// temporary storage from the stream-ordered pool.  Returns a GP_* status.
int gp_internal_radix_sort_pairs_u32(const uint32_t *keys_in, uint32_t *keys_out, const uint32_t *vals_in,
                                     uint32_t *vals_out, size_t n, int end_bit, hipStream_t s,
                                     std::string *error);

namespace {

typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kBlock = 256;
// A block-stride grid of this many blocks per CU saturates HBM on 256 CUs
// while keeping launch cost flat for any problem size.
constexpr int kBlocksPerCU = 8;
constexpr int kMaxBucketsPerLaunch = 8;

thread_local std::string g_last_error;

int set_error(int code, const std::string &msg) {
  g_last_error = msg;
  return code;
}

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

int num_cus() {
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

size_t grid_cap() { return (size_t)num_cus() * kBlocksPerCU; }

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
// on the same stream wrote: the unplanned calls' steady state (§ "Device-built
// plans" below) launches both the cached plan and the op-order fallback right
// behind the index check, and exactly one of them does any work, with no host
// round trip.  `word` holds the generation of the last call whose check found
// the index changed; this call's generation is `gen`.  A kernel's GATED = true
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

int launch_bucket_sum(float *out, const float *in, const float *const *bk,
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
// HBM probe (measurement only): one buffer streamed once, read-only, with
// 16-B non-temporal loads, 4 block-strides in flight per thread, 2 blocks per
// CU -- the fastest of 16 shapes (U 4-16, 1-8 blocks per CU, nt or plain):
// 6.3-7.1 TB/s (profiles/r02/tune/probe_tune*.txt).  bench.py times it beside
// the reduction, and a write-only stream beside it, to give each kernel's
// bytes a same-box two-rate model: t = read_bytes / read_rate +
// write_bytes / write_rate.
// ---------------------------------------------------------------------------
constexpr int kProbeU = 4;
}  // namespace
// The read probe's sink: never the probed buffer.  External linkage on purpose:
// a sink with internal linkage that nothing reads lets the compiler drop the
// store, then every load feeding it (the kernel compiled to an empty body and
// the "read rate" came out at 674 TB/s in profiles/r03/full/bench_default.json).
__device__ float gp_probe_sink[64];
namespace {

__global__ __launch_bounds__(kBlock) void hbm_read_probe_kernel(const f4 *__restrict__ in, size_t n4) {
  const size_t tile = (size_t)kBlock * kProbeU;
  const size_t stride = (size_t)gridDim.x * tile;
  f4 acc = f4(0.0f);
  size_t base = (size_t)blockIdx.x * tile + threadIdx.x;
  for (; base + (kProbeU - 1) * kBlock < n4; base += stride) {
    f4 v[kProbeU];
#pragma unroll
    for (int u = 0; u < kProbeU; ++u) v[u] = __builtin_nontemporal_load(in + base + u * kBlock);
#pragma unroll
    for (int u = 0; u < kProbeU; ++u) acc += v[u];
  }
  for (int u = 0; u < kProbeU; ++u)
    if (base + u * kBlock < n4) acc += __builtin_nontemporal_load(in + base + u * kBlock);
  // data-dependent, practically never true: keeps every load live
  if (acc.x + acc.y + acc.z + acc.w == -1234.5f) gp_probe_sink[blockIdx.x % 64] = acc.x;
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

int check_segments(const gp_row_segments *t, size_t row_size, bool *aligned) {
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

// ---------------------------------------------------------------------------
// Row plans: a scatter DoubleIndex compiled once (libgeeps' indexes are fixed
// at FinishVirtualIteration, clientlib-viter.cpp:817-883).
//
// The plan visits the rows in destination (id1) order, offsets applied.  That
// is bit-neutral because destinations are distinct: every destination row
// receives exactly the same adds whatever order the rows are visited in.
//  * Dense runs: maximal runs in which id0 and id1 both step by one and every
//    row is clear of num_vals_limit are plain ranges y[y0 .. y0 + L*W) (+)=
//    x[x0 .. x0 + L*W).  Runs of at least kDenseRunBytes go to the phase-
//    separated sum kernels (one bucket; the fused init through their ZIN
//    form), which read no index and, unlike any single-pass form, keep their
//    rate on every allocation: over 10 fresh allocations the add ran 76.5-
//    80.9 % of 8 TB/s this way against 63-80 % through the wave-map kernel,
//    which fell to 63-69 % on 7 of them (profiles/r02/tune/rowop_alloc*.txt).
//    libgeeps assigns cache rows in first-access order, so an op's rows are
//    typically one run per channel.
//  * The other rows keep a device index, sorted by id1, for the wave-map
//    kernel with non-temporal oplog accesses and one resident round of blocks:
//    the read-modify-write side walks the oplog front to back like the
//    gather's write side: 77-79 % for a random permutation, against 63-65 %
//    for the same index in op order through row_op_kernel (plan_tune*.txt).
// ---------------------------------------------------------------------------
// A dense run launches 1-3 kernels; below 4 MiB (the phased form's smallest
// shard) the row kernel moves it without the launches.
constexpr size_t kDenseRunBytes = 4u << 20;

struct RowRun {
  uint64_t x_row, y_row, rows;  // offsets applied
};

}  // namespace

struct gp_row_plan_s {
  size_t num_rows = 0, row_size = 0, limit = 0;
  bool gather = false;  // a gather plan (y[id0] = x[id1]); else a scatter plan
  std::vector<RowRun> dense;
  size_t dense_rows = 0;
  // device, offsets applied, ascending destination (scatter: id1, gather: id0)
  gp_double_index *residual = nullptr;
  size_t residual_rows = 0;
  // Repeated destinations: layer k holds each destination's (k+1)-th
  // occurrence in op order (device, ascending destination), run after the
  // layers before it, so a repeated row receives its adds in op order.
  struct Layer {
    gp_double_index *index = nullptr;
    size_t rows = 0;
  };
  std::vector<Layer> repeats;
  size_t repeat_rows = 0;
  int device = 0;
};

namespace {

// Scatter plans (y[id1] (+)= x[id0], the limit on the source x) sort by id1;
// gather plans (y[id0] = x[id1], assign_rows_to_double_index, the limit on
// the destination y) sort by id0.  Either way the limit guards the id0 side
// and the destination must not repeat.
int build_row_plan(gp_row_plan_s *p, const gp_double_index *host_index, size_t n,
                   gp_double_index off) {
  using Layer = gp_row_plan_s::Layer;
  const size_t W = p->row_size;
  const bool g = p->gather;
  std::vector<gp_double_index> rows(n);
  for (size_t r = 0; r < n; ++r)
    rows[r] = gp_double_index{host_index[r].id0 + off.id0, host_index[r].id1 + off.id1};
  auto dst = [g](const gp_double_index &d) { return g ? d.id0 : d.id1; };
  // stable: a repeated destination keeps its occurrences in op order
  std::stable_sort(rows.begin(), rows.end(), [&](const gp_double_index &a, const gp_double_index &b) {
    return dst(a) < dst(b);
  });
  // A destination listed k + 1 times: its first occurrence stays in `rows`
  // (distinct destinations), the later ones go to repeat layers 1..k.  The
  // reference's channel check (range == count, clientlib-viter.cpp:869-873)
  // admits such an index, e.g. cache rows {0, 0, 2}; its CPU twin
  // (row-op-util.hpp:121-139) adds the repeats in op order, its GPU kernel races
  // on them (row-op-util.cu:109-125).  The layers reproduce the CPU order: each
  // layer has distinct destinations and runs after the one before it.
  std::vector<std::vector<gp_double_index>> layers;
  {
    size_t w = 0, k = 0;
    for (size_t r = 0; r < n; ++r) {
      k = (r > 0 && dst(rows[r]) == dst(rows[r - 1])) ? k + 1 : 0;
      if (k == 0) {
        rows[w++] = rows[r];
      } else {
        if (layers.size() < k) layers.resize(k);
        layers[k - 1].push_back(rows[r]);
      }
    }
    rows.resize(w);
    n = w;
  }
  for (auto &l : layers) {
    Layer d;
    d.rows = l.size();
    GP_HIP_TRY(hipMalloc(&d.index, l.size() * sizeof(gp_double_index)));
    p->repeats.push_back(d);  // owned by the plan from here (freed on any error)
    GP_HIP_TRY(hipMemcpy(d.index, l.data(), l.size() * sizeof(gp_double_index), hipMemcpyHostToDevice));
    p->repeat_rows += l.size();
  }
  auto whole = [&](const gp_double_index &d) { return (d.id0 + 1) * W <= p->limit; };
  const size_t min_rows = std::max<size_t>(1, kDenseRunBytes / (W * sizeof(float)));
  std::vector<gp_double_index> rest;
  for (size_t a = 0; a < n;) {
    size_t b = a + 1;
    if (whole(rows[a]))
      while (b < n && whole(rows[b]) && rows[b].id0 == rows[b - 1].id0 + 1 &&
             rows[b].id1 == rows[b - 1].id1 + 1)
        ++b;
    if (whole(rows[a]) && b - a >= min_rows) {
      p->dense.push_back(g ? RowRun{rows[a].id1, rows[a].id0, b - a}
                           : RowRun{rows[a].id0, rows[a].id1, b - a});
      p->dense_rows += b - a;
    } else {
      rest.insert(rest.end(), rows.begin() + a, rows.begin() + b);
    }
    a = b;
  }
  p->residual_rows = rest.size();
  if (!rest.empty()) {
    GP_HIP_TRY(hipMalloc(&p->residual, rest.size() * sizeof(gp_double_index)));
    GP_HIP_TRY(hipMemcpy(p->residual, rest.data(), rest.size() * sizeof(gp_double_index),
                         hipMemcpyHostToDevice));
  }
  return GP_OK;
}

// OP kAddFrom: y += x over the plan's rows; kInitFrom: y = 0.0f + x (0.0f past
// the limit), as gp_scatter_add_rows / gp_scatter_init_rows with the plan's
// index, offset and limit.
int check_plan(const gp_row_plan_s *p, bool gather) {
  if (!p) return set_error(GP_ERR_INVALID, "null row plan");
  if (p->gather != gather)
    return set_error(GP_ERR_INVALID, gather ? "a scatter row plan passed to a gather"
                                            : "a gather row plan passed to a scatter");
  if (p->residual_rows || p->repeat_rows) {
    int dev = -1;
    GP_HIP_TRY(hipGetDevice(&dev));
    if (dev != p->device)
      return set_error(GP_ERR_INVALID, "row plan used on another device than it was built on");
  }
  return GP_OK;
}

template <int OP>
int launch_planned(float *y, const float *x, const gp_row_plan_s *p, hipStream_t s) {
  const int rc0 = check_plan(p, false);
  if (rc0 != GP_OK) return rc0;
  if (p->num_rows == 0) return GP_OK;
  const size_t W = p->row_size;
  for (const RowRun &r : p->dense) {
    BucketPtrs b = {};
    b.p[0] = x + r.x_row * W;
    float *yr = y + r.y_row * W;
    const int rc = OP == kAddFrom ? launch_bucket_sum_nb<1>(yr, yr, b, r.rows * W, s)
                                  : launch_bucket_sum_nb<1, true>(yr, nullptr, b, r.rows * W, s);
    if (rc != GP_OK) return rc;
  }
  if (p->residual_rows) {
    const int rc = launch_row_op<OP>(y, x, p->residual, p->residual_rows, gp_double_index{0, 0}, W,
                                     p->limit, s, /*sorted=*/true);
    if (rc != GP_OK) return rc;
  }
  // later occurrences of repeated destinations: added in op order (the init's
  // first occurrence zeroed the row; the rest add to it)
  for (const auto &l : p->repeats) {
    const int rc = launch_row_op<kAddFrom>(y, x, l.index, l.rows, gp_double_index{0, 0}, W, p->limit, s,
                                           /*sorted=*/true);
    if (rc != GP_OK) return rc;
  }
  return GP_OK;
}

// A gather plan: y[id0] = x[id1] over the plan's rows, x flat (xs == nullptr)
// or a segmented cache.  Dense runs are plain copies through the bucket-sum
// kernels with no bucket (NB = 0: the sweep's 64-MiB chunks, then the
// tile-major and mixed forms), split where a run crosses a segment boundary;
// the residual rows through the gather row kernels, in destination order.
int launch_gather_planned(float *y, const float *x, const gp_row_segments *xs,
                          const gp_row_plan_s *p, hipStream_t s) {
  const int rc0 = check_plan(p, true);
  if (rc0 != GP_OK) return rc0;
  if (p->num_rows == 0) return GP_OK;
  bool seg_aligned = false;
  if (xs) {
    const int rc = check_segments(xs, p->row_size, &seg_aligned);
    if (rc != GP_OK) return rc;
  }
  const size_t W = p->row_size;
  const BucketPtrs none = {};
  for (const RowRun &r : p->dense) {
    uint64_t row = r.x_row, left = r.rows;  // source (cache) rows still to copy
    float *yr = y + r.y_row * W;
    while (left) {
      const float *src = nullptr;
      uint64_t take = left;
      if (!xs) {
        src = x + row * W;
      } else {
        uint32_t i = 0;  // the segment holding `row`: the last one starting at or before it
        while (i + 1 < xs->count && xs->first_row[i + 1] <= row) ++i;
        src = xs->base[i] + (row - xs->first_row[i]) * W;
        if (i + 1 < xs->count) take = std::min<uint64_t>(take, xs->first_row[i + 1] - row);
      }
      const int rc = launch_bucket_sum_nb<0>(yr, src, none, take * W, s);
      if (rc != GP_OK) return rc;
      yr += take * W;
      row += take;
      left -= take;
    }
  }
  // the residual, then later occurrences of repeated destinations (assigned in
  // op order: the last one listed wins, as in the CPU twin's loop)
  std::vector<gp_row_plan_s::Layer> parts;
  if (p->residual_rows) parts.push_back({p->residual, p->residual_rows});
  parts.insert(parts.end(), p->repeats.begin(), p->repeats.end());
  for (const auto &l : parts) {
    const int rc = xs ? launch_row_op_seg<kAssignTo, kSegX>(y, xs, l.index, l.rows, gp_double_index{0, 0},
                                                             W, p->limit, s)
                      : launch_row_op<kAssignTo>(y, x, l.index, l.rows, gp_double_index{0, 0}, W,
                                                 p->limit, s, /*sorted=*/true);
    if (rc != GP_OK) return rc;
  }
  return GP_OK;
}

// ---------------------------------------------------------------------------
// Device-built plans for the unplanned calls (gp_scatter_add_rows,
// gp_scatter_init_rows, gp_gather_rows): the reference's own binding passes a
// device DoubleIndex on every call (add_rows_from_double_index_gpu,
// row-op-util.cu:127-142, synchronous at :141), with no host copy to compile a
// gp_row_plan from.  A large call therefore plans itself on the device:
//  1. index_scan_kernel reads the index once (16 B per row) and writes, per
//     64-entry tile, whether it is dense (id0 and id1 both step by one, every
//     row clear of num_vals_limit), whether it continues the tile before, and
//     whether its destinations ascend; the first entry of every tile that
//     starts a dense run; the largest destination row.  When the call's index
//     was planned before (the plan cache, below), it also compares every entry
//     with the copy kept then.
//  2. One D2H of that summary and a stream sync (the reference's call syncs
//     too); the host turns it into runs, as build_row_plan does.
//  3. Dense runs of at least kDenseRunBytes go to the phase-separated sum
//     kernels (1 bucket, the zero-input form, the copy), as in a row plan.
//  4. The other rows (the residual) go to the row kernels.  A scatter-add's or
//     init's residual whose destinations do not ascend is a random
//     read-modify-write of y in op order (~66 % of 8 TB/s; a plan's
//     destination-sorted residual runs ~76 %).  Sorting it costs more than it
//     saves in one call (a radix sort of 8 M pairs ~0.3 ms; coarse binning
//     does not recover the locality: DESIGN.md §5), but the reference reuses
//     each op's DoubleIndex every clock.  So the first call with an index runs
//     such a residual in op order and keeps a copy of the index; the second
//     call with the same index -- same pointer, size, offsets, row size and
//     limit, and entry for entry the same content, which the scan checks
//     against the copy -- builds the destination-sorted residual (a hipCUB
//     radix sort, gp_sort.hip) and runs it.  Later calls (the steady state)
//     skip the scan and the host round trip: index_verify_kernel compares the
//     index with the copy and, if any entry changed, writes the call's
//     generation into a gate word; the cached dense runs and sorted residual
//     are launched behind it gated to run only if nothing changed, and the
//     op-order form of the whole call gated to run only if something did
//     (Gate, the GATED kernel forms).  No D2H, no stream sync: the call is as
//     asynchronous as a planned one.  The check also sets a host-visible word,
//     which a later call reads to drop the stale entry and plan afresh.
//     An index that changes every call costs one copy per call, no sort.  Visiting rows in destination order is bit-neutral under
//     the call's precondition (distinct destinations).
// Calls below g_analyze_min_bytes (gp_set_unplanned_min_bytes) skip all this.
// ---------------------------------------------------------------------------
constexpr int kScanGroupTiles = 64;  // tiles of 64 entries per scan word group
constexpr int kScanWaveTiles = 16;   // tiles per wave (17 loads in flight)
constexpr int kMaxRunStarts = 512;   // run-start entries the scan records
constexpr int kMaxDeviceRuns = 32;   // dense runs a call sweeps (the longest)
constexpr size_t kSortMinBytes = 16u << 20;       // smaller residuals keep op order
constexpr size_t kInvSpread = 4;  // an inverse map may span up to 4 x its rows (+ 1 Mi)
std::atomic<size_t> g_plan_cache_bytes{4ull << 30};  // device memory of cached plans (LRU)
constexpr size_t kPlanCacheEntries = 256;

struct ScanHeader {
  unsigned int n_starts;
  unsigned int mismatches;  // blocks that saw an entry differ from the cached copy
  uint64_t pad;
};
struct RunStart {
  uint64_t tile, from, to;
};
// workspace: [ScanHeader][RunStart x kMaxRunStarts][4 words per group of 64
// tiles: dense, continues, ascends (bit k = tile 64 g + k), largest destination]
constexpr size_t kScanWordsOff = sizeof(ScanHeader) + sizeof(RunStart) * kMaxRunStarts;
constexpr int kScanWords = 4;

std::atomic<size_t> g_analyze_min_bytes{64u << 20};

int radix_sort_pairs_u32(const uint32_t *ki, uint32_t *ko, const uint32_t *vi, uint32_t *vo, size_t n, int end_bit,
                         hipStream_t s) {
  std::string err;
  const int rc = gp_internal_radix_sort_pairs_u32(ki, ko, vi, vo, n, end_bit, s, &err);
  return rc == GP_OK ? GP_OK : set_error(rc, err);
}

__device__ __forceinline__ uint64_t lane_u64(uint64_t v, int lane) {  // v of `lane`, wave-uniform
  const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, lane);
  const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane);
  return ((uint64_t)hi << 32) | lo;
}

// One block (4 waves) per group of 64 tiles (4096 entries); each wave takes 16
// tiles with all 17 of its loads (the tile before its first, then its own) in
// flight at once.  A tile is dense when every lane's endpoints are lane 0's
// plus the lane number (lane 0's and lane 63's values are read into scalar
// registers, no LDS traffic); only the ascending test needs a lane shuffle.
// No global atomics on the common path (a per-group word carries the group's
// largest destination).
template <int OP, bool CMP>
__global__ __launch_bounds__(kBlock) void index_scan_kernel(const gp_double_index *__restrict__ idx, size_t n,
                                                            uint64_t off0, uint64_t off1, size_t row_size,
                                                            size_t limit, const gp_double_index *__restrict__ cached,
                                                            char *__restrict__ ws) {
  static_assert(kScanWaveTiles * (kBlock / 64) == kScanGroupTiles, "a block covers one word group");
  ScanHeader *hdr = reinterpret_cast<ScanHeader *>(ws);
  RunStart *starts = reinterpret_cast<RunStart *>(ws + sizeof(ScanHeader));
  uint64_t *words = reinterpret_cast<uint64_t *>(ws + kScanWordsOff);
  __shared__ uint64_t part[kScanWords][kBlock / 64];
  const int wl = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const size_t tiles = (n + 63) / 64;
  const size_t groups = (tiles + kScanGroupTiles - 1) / kScanGroupTiles;
  for (size_t g = blockIdx.x; g < groups; g += gridDim.x) {
    const size_t t0 = g * kScanGroupTiles + (size_t)wv * kScanWaveTiles;  // this wave's first tile
    uint64_t f[kScanWaveTiles + 1], to[kScanWaveTiles + 1];
    bool whole[kScanWaveTiles + 1];
    bool differs = false;
    // every load unconditional (addresses clamped into the index, results
    // masked after), so all of a wave's loads are in flight before the first wait
    gp_double_index raw[kScanWaveTiles + 1], cp[kScanWaveTiles + 1];
#pragma unroll
    for (int k = 0; k <= kScanWaveTiles; ++k) {  // k = 0: the tile before t0
      const size_t e = t0 + k >= 1 ? (t0 + k - 1) * 64 + wl : 0;
      const size_t ec = e < n ? e : n - 1;
      raw[k] = idx[ec];
      if (CMP && k > 0) cp[k] = cached[ec];
    }
#pragma unroll
    for (int k = 0; k <= kScanWaveTiles; ++k) {  // selects, no branches: the loads stay hoisted
      const size_t e = t0 + k >= 1 ? (t0 + k - 1) * 64 + wl : 0;
      const bool live = (t0 + k >= 1) & (e < n);
      uint64_t a, b;
      row_endpoints<OP>(raw[k], off0, off1, a, b);
      const bool wh = ((OP == kAssignTo ? b : a) + 1) * row_size <= limit;
      whole[k] = live & wh;
      f[k] = live ? a : 0;
      to[k] = live ? b : 0;
      if (CMP && k > 0) differs |= live & ((cp[k].id0 != raw[k].id0) | (cp[k].id1 != raw[k].id1));
    }
    auto tile_dense = [&](int k) {  // every lane whole and lane 0 + lane
      const uint64_t b0 = lane_u64(f[k], 0), b1 = lane_u64(to[k], 0);
      return __all(whole[k] && f[k] == b0 + (uint64_t)wl && to[k] == b1 + (uint64_t)wl);
    };
    bool prev_dense = t0 >= 1 && tile_dense(0);
    uint64_t pf = lane_u64(f[0], 63), pt = lane_u64(to[0], 63);  // the entry before the tile
    uint32_t wd = 0, wc = 0, wa = 0;
    uint64_t mx = 0;
#pragma unroll
    for (int k = 1; k <= kScanWaveTiles; ++k) {
      const size_t t = t0 + k - 1;
      const size_t e = t * 64 + wl;
      const bool live = e < n;
      const uint64_t f0 = lane_u64(f[k], 0), to0 = lane_u64(to[k], 0);
      const bool dense = t < tiles && tile_dense(k);
      const bool cont = t > 0 && f0 == pf + 1 && to0 == pt + 1;  // wave-uniform
      const uint64_t lt = shfl64(to[k], (wl + 63) & 63);
      const bool asc = __all(!live || e == 0 || to[k] > (wl == 0 ? pt : lt));
      if (live && to[k] > mx) mx = to[k];
      wd |= (dense ? 1u : 0u) << (k - 1);
      wc |= (cont ? 1u : 0u) << (k - 1);
      wa |= (asc ? 1u : 0u) << (k - 1);
      if (dense && !(cont && prev_dense) && wl == 0) {
        const unsigned slot = atomicAdd(&hdr->n_starts, 1u);
        if (slot < (unsigned)kMaxRunStarts) starts[slot] = RunStart{t, f0, to0};
      }
      prev_dense = dense;
      pf = lane_u64(f[k], 63);
      pt = lane_u64(to[k], 63);
    }
    __shared__ unsigned block_differs;
    if (CMP && threadIdx.x == 0) block_differs = 0;
    for (int o = 32; o > 0; o >>= 1) {
      const uint64_t v = shfl64(mx, (wl + o) & 63);
      mx = v > mx ? v : mx;
    }
    if (wl == 0) {
      part[0][wv] = (uint64_t)wd << (wv * kScanWaveTiles);
      part[1][wv] = (uint64_t)wc << (wv * kScanWaveTiles);
      part[2][wv] = (uint64_t)wa << (wv * kScanWaveTiles);
      part[3][wv] = mx;
    }
    __syncthreads();
    if (CMP && __any(differs) && wl == 0) atomicOr(&block_differs, 1u);  // one global atomic per block, below
    __syncthreads();
    if (CMP && threadIdx.x == 0 && block_differs) atomicAdd(&hdr->mismatches, 1u);
    if (threadIdx.x < kScanWords) {
      uint64_t w = 0;
      for (int v = 0; v < kBlock / 64; ++v)
        w = threadIdx.x == 3 ? (part[3][v] > w ? part[3][v] : w) : (w | part[threadIdx.x][v]);
      words[kScanWords * g + threadIdx.x] = w;
    }
    __syncthreads();
  }
}

// The steady state's check of a planned index seen again: whether every entry
// still equals the kept copy (no tile analysis).  Two forms of the copy:
//   full     the 16-B entries (32 B read per entry);
//   compact  when the kept index has id0 = base0 + position and id1 < 2^32
//            (the reference's op buffers list their rows in order: id0 is
//            the position, clientlib-viter.cpp:841), only id1 as 4 B: the
//            check reads 20 B per entry and still compares all 128 bits.
// Each thread holds 4 entries' loads in flight.  A difference puts this
// call's generation into the call's gate word (the gated launches behind it
// read it) and into the entry's host-visible word (the next call drops the
// entry), through flag_once.
constexpr int kCmpPerThread = 4;
constexpr unsigned kGateSlots = 64;  // gate words per entry: calls in flight on one entry

// A launch's finding (an index changed, a map unsound, a copy not compact):
// `dev_word` := v for the kernels behind it, and `host_word` := v for the
// host, at most one atomic per block and one host write per launch -- the
// block whose exchange changed the device word writes it.  (A store per wave
// to the host-visible word crosses the bus each time: a launch that found
// differences everywhere took 1.06 ms instead of 25 us.)  Every thread of the
// block calls it: `hit` is reduced over the block.
__device__ __forceinline__ void flag_once(bool hit, unsigned *dev_word, unsigned *host_word, unsigned v) {
  if (!__syncthreads_or(hit) || threadIdx.x != 0) return;
  if (__hip_atomic_exchange(dev_word, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != v)
    __hip_atomic_store(host_word, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <bool COMPACT>
__device__ __forceinline__ void index_verify(const gp_double_index *__restrict__ idx, const void *__restrict__ kept,
                                             size_t n, const uint64_t *__restrict__ base0_word,
                                             unsigned *__restrict__ gate_word, unsigned *__restrict__ host_word,
                                             unsigned gen, bool sticky) {
  const size_t step = (size_t)gridDim.x * kBlock * kCmpPerThread;
  const uint64_t base0 = COMPACT ? *base0_word : 0;
  bool differs = sticky;
  for (size_t base = (size_t)blockIdx.x * kBlock * kCmpPerThread + threadIdx.x; base < n; base += step) {
    gp_double_index a[kCmpPerThread], b[kCmpPerThread];
    uint32_t c[kCmpPerThread];
#pragma unroll
    for (int k = 0; k < kCmpPerThread; ++k) {  // clamped, unconditional: all loads in flight
      const size_t e = base + (size_t)k * kBlock;
      const size_t ec = e < n ? e : n - 1;
      a[k] = idx[ec];
      if constexpr (COMPACT)
        c[k] = static_cast<const uint32_t *>(kept)[ec];
      else
        b[k] = static_cast<const gp_double_index *>(kept)[ec];
    }
#pragma unroll
    for (int k = 0; k < kCmpPerThread; ++k) {
      if constexpr (COMPACT) {
        const size_t ec = base + (size_t)k * kBlock < n ? base + (size_t)k * kBlock : n - 1;
        differs |= (a[k].id0 != base0 + ec) | (a[k].id1 != (uint64_t)c[k]);
      } else {
        differs |= (a[k].id0 != b[k].id0) | (a[k].id1 != b[k].id1);
      }
    }
  }
  flag_once(differs, gate_word, host_word, gen);
}

// FORM 0: against the full copy, 1: the compact copy, 2: whichever the
// entry has, by compact_copy_kernel's `broken` flag (read on the device: the
// host may not know it yet, and an entry may keep no full copy of a compact
// index, copy_if_broken_kernel).
template <int FORM>
__global__ __launch_bounds__(kBlock) void index_verify_kernel(const gp_double_index *__restrict__ idx,
                                                              const gp_double_index *__restrict__ full,
                                                              const uint32_t *__restrict__ compact, size_t n,
                                                              const uint64_t *__restrict__ base0_word,
                                                              unsigned *__restrict__ gate_word,
                                                              unsigned *__restrict__ host_word, unsigned gen,
                                                              const unsigned *__restrict__ broken,
                                                              const unsigned *__restrict__ unsound) {
  bool use_compact = FORM == 1;
  if constexpr (FORM == 2) use_compact = __hip_atomic_load(broken, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
  // an entry whose inverse map was found unsound when it was built
  // (inverse_scatter_kernel / inverse_count_kernel set the sticky word): every
  // later call treats its index as changed, so no gated launch walks the map,
  // however soon after the build it was queued
  const bool sticky = __hip_atomic_load(unsound, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  if (use_compact)
    index_verify<true>(idx, compact, n, base0_word, gate_word, host_word, gen, sticky);
  else
    index_verify<false>(idx, full, n, base0_word, gate_word, host_word, gen, sticky);
}

// The compact copy of an index (built with the plan: on the first call for an
// inverse or ranges plan, on the second with a sorted residual): id1 as 4 B
// per entry and base0 = id0 of entry 0; `host_broken` and
// `dev_broken` (a device word the next kernels read) set
// when the index is not of that shape (then the full copy stays in use).
__global__ __launch_bounds__(kBlock) void compact_copy_kernel(const gp_double_index *__restrict__ idx, size_t n,
                                                              uint32_t *__restrict__ id1_out,
                                                              uint64_t *__restrict__ base0_out,
                                                              unsigned *__restrict__ host_broken,
                                                              unsigned *__restrict__ dev_broken) {
  const uint64_t base0 = idx[0].id0;
  if (blockIdx.x == 0 && threadIdx.x == 0) *base0_out = base0;
  bool bad = false;
  const size_t stride = (size_t)gridDim.x * kBlock;
  for (size_t e = (size_t)blockIdx.x * kBlock + threadIdx.x; e < n; e += stride) {
    const gp_double_index v = idx[e];
    bad |= (v.id0 != base0 + e) | ((v.id1 >> 32) != 0);
    id1_out[e] = (uint32_t)v.id1;
  }
  flag_once(bad, dev_broken, host_broken, 1u);
}

// The full copy of an index whose steady state checks the compact copy:
// written only if compact_copy_kernel (earlier on the stream) found the index
// not of the compact shape, the one case index_verify_kernel<false> reads it.
__global__ __launch_bounds__(kBlock) void copy_if_broken_kernel(const gp_double_index *__restrict__ idx, size_t n,
                                                                gp_double_index *__restrict__ out,
                                                                const unsigned *__restrict__ broken) {
  if (__hip_atomic_load(broken, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
  const size_t stride = (size_t)gridDim.x * kBlock;
  for (size_t e = (size_t)blockIdx.x * kBlock + threadIdx.x; e < n; e += stride) out[e] = idx[e];
}

// Residual rows of a call: up to kMaxDeviceRuns + 1 entry ranges, passed by
// value; `pre[i]` = rows in ranges before i.
struct EntryRanges {
  uint32_t count;
  uint64_t lo[kMaxDeviceRuns + 1], hi[kMaxDeviceRuns + 1], pre[kMaxDeviceRuns + 2];
};

__device__ __forceinline__ size_t range_entry(const EntryRanges &r, size_t k) {
  uint32_t i = 0;
  while (i + 1 < r.count && r.pre[i + 1] <= k) ++i;
  return r.lo[i] + (k - r.pre[i]);
}

// Sort keys (destination rows) and values (entry positions) of the residual.
template <int OP>
__global__ __launch_bounds__(kBlock) void residual_keys_kernel(const gp_double_index *__restrict__ idx, EntryRanges rr,
                                                               uint64_t off0, uint64_t off1, uint32_t *__restrict__ key,
                                                               uint32_t *__restrict__ val) {
  const size_t total = rr.pre[rr.count];
  const size_t stride = (size_t)gridDim.x * kBlock;
  for (size_t k = (size_t)blockIdx.x * kBlock + threadIdx.x; k < total; k += stride) {
    const size_t e = range_entry(rr, k);
    uint64_t f, t;
    row_endpoints<OP>(idx[e], off0, off1, f, t);
    key[k] = (uint32_t)t;
    val[k] = (uint32_t)e;
  }
}

// The residual's entries in sorted order, offsets applied (a scatter plan's
// residual: {from, to}).
template <int OP>
__global__ __launch_bounds__(kBlock) void residual_gather_kernel(const gp_double_index *__restrict__ idx,
                                                                 const uint32_t *__restrict__ pos, size_t total,
                                                                 uint64_t off0, uint64_t off1,
                                                                 gp_double_index *__restrict__ out) {
  const size_t stride = (size_t)gridDim.x * kBlock;
  for (size_t k = (size_t)blockIdx.x * kBlock + threadIdx.x; k < total; k += stride) {
    uint64_t f, t;
    row_endpoints<OP>(idx[pos[k]], off0, off1, f, t);
    out[k] = gp_double_index{f, t};
  }
}

// The inverse map of a call's residual (the unplanned calls' inverse plan):
// inv[to] = entry << 32 | from, offsets applied, over destination rows 0 ..
// D - 1 (~0 = no residual row goes there; the caller fills it first).  Plain
// stores: destinations are distinct by the calls' precondition, and
// inverse_count_kernel then proves it (a repeated destination leaves fewer
// listed rows than residual entries).  A source row past 2^32 (a 4-B field)
// or a repeated destination stores this call's generation into the gate word
// and the host-visible word: the map is then unsound, the gated op-order
// launches run instead, and the next call drops the plan.  (A compare-and-swap
// scatter that checks as it goes measured 2.5x the plain scatter.)
template <int OP>
__global__ __launch_bounds__(kBlock) void inverse_scatter_kernel(const gp_double_index *__restrict__ idx, EntryRanges rr,
                                                                 uint64_t off0, uint64_t off1,
                                                                 uint64_t *__restrict__ inv,
                                                                 unsigned *__restrict__ gate_word,
                                                                 unsigned *__restrict__ host_word, unsigned gen,
                                                                 unsigned *__restrict__ unsound) {
  const size_t total = rr.pre[rr.count];
  const size_t stride = (size_t)gridDim.x * kBlock;
  bool bad = false;
  for (size_t k = (size_t)blockIdx.x * kBlock + threadIdx.x; k < total; k += stride) {
    const size_t e = range_entry(rr, k);
    uint64_t f, t;
    row_endpoints<OP>(idx[e], off0, off1, f, t);
    bad |= (f >> 32) != 0;
    inv[t] = ((uint64_t)e << 32) | (f & 0xffffffffu);
  }
  if (bad) __hip_atomic_store(unsound, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // (rare)
  flag_once(bad, gate_word, host_word, gen);
}

// Whether the inverse map lists exactly `expected` rows (the residual's
// entries): one sequential pass over it (16 loads in flight per thread), a
// block sum, one atomic add per block (a launch of about one block per CU:
// per-wave atomics on one address measured 254 us); the last block to finish
// compares and, on a shortfall (a repeated destination), marks the map
// unsound as inverse_scatter_kernel does.
constexpr int kCountPerThread = 16;
__global__ __launch_bounds__(kBlock) void inverse_count_kernel(const uint64_t *__restrict__ inv, size_t rows,
                                                               uint64_t expected, unsigned long long *counters,
                                                               unsigned *__restrict__ gate_word,
                                                               unsigned *__restrict__ host_word, unsigned gen,
                                                               unsigned *__restrict__ unsound) {
  const size_t step = (size_t)gridDim.x * kBlock * kCountPerThread;
  unsigned listed = 0;
  for (size_t base = (size_t)blockIdx.x * kBlock * kCountPerThread + threadIdx.x; base < rows; base += step) {
    uint64_t v[kCountPerThread];
#pragma unroll
    for (int k = 0; k < kCountPerThread; ++k) {
      const size_t r = base + (size_t)k * kBlock;
      v[k] = r < rows ? inv[r] : ~0ull;
    }
#pragma unroll
    for (int k = 0; k < kCountPerThread; ++k) listed += v[k] != ~0ull;
  }
  for (int o = 32; o > 0; o >>= 1) listed += __shfl_xor(listed, o, 64);
  __shared__ unsigned wave_sum[kBlock / 64];
  if ((threadIdx.x & 63) == 0) wave_sum[threadIdx.x / 64] = listed;
  __syncthreads();
  if (threadIdx.x != 0) return;
  unsigned long long block = 0;
  for (int w = 0; w < kBlock / 64; ++w) block += wave_sum[w];
  __hip_atomic_fetch_add(&counters[0], block, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (__hip_atomic_fetch_add(&counters[1], 1ull, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) != gridDim.x - 1ull)
    return;
  if (__hip_atomic_load(&counters[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != expected) {
    __hip_atomic_store(unsound, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(gate_word, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(host_word, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Thread-local pinned landing buffer for the scan summary (a call's D2H is
// complete, after its sync, before the same thread issues the next).
struct PinnedScratch {
  void *p = nullptr;
  size_t bytes = 0;
  ~PinnedScratch() {
    if (p) (void)hipHostFree(p);
  }
  void *get(size_t need) {
    if (need > bytes) {
      if (p) (void)hipHostFree(p);
      p = nullptr;
      bytes = 0;
      if (hipHostMalloc(&p, need, hipHostMallocDefault) != hipSuccess) return nullptr;
      bytes = need;
    }
    return p;
  }
};
thread_local PinnedScratch g_scan_landing;

// The workspaces come from the device's default stream-ordered pool
// (hipMallocAsync / hipFreeAsync, safe across streams); keep what it holds
// instead of returning it to the driver at every sync (release threshold 0
// by default), so a call's allocations are pool hits after the first.
std::atomic<bool> g_pool_kept[kMaxDevices];

void keep_pool_memory() {
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return;
  if (g_pool_kept[dev].exchange(true)) return;
  hipMemPool_t pool;
  if (hipDeviceGetDefaultMemPool(&pool, dev) != hipSuccess) return;
  uint64_t keep = UINT64_MAX;
  (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
}

// ---- the plan cache --------------------------------------------------------
struct PlanKey {
  int device, op;
  uintptr_t index;
  size_t n, row_size, limit;
  uint64_t off0, off1;
  bool operator==(const PlanKey &o) const {
    return device == o.device && op == o.op && index == o.index && n == o.n && row_size == o.row_size &&
           limit == o.limit && off0 == o.off0 && off1 == o.off1;
  }
};

// Device memory of a plan-cache entry, from the device's stream-ordered pool
// (hipMallocAsync on the building call's stream: the pool keeps what it was
// given, keep_pool_memory, so a first call's allocations do not stall it).
// Freed only after the device is idle (~CachedPlan waits for it first),
// back to the pool.
struct DevBuf {
  void *p = nullptr;
  int device = 0;
  DevBuf(size_t bytes, int dev, hipStream_t s, int *rc) : device(dev) {
    *rc = hipMallocAsync(&p, bytes, s) == hipSuccess ? GP_OK : set_error(GP_ERR_HIP, "plan cache hipMallocAsync");
  }
  ~DevBuf() {
    if (!p) return;
    int cur = -1;
    (void)hipGetDevice(&cur);
    if (cur != device) (void)hipSetDevice(device);
    (void)hipFreeAsync(p, nullptr);
    if (cur >= 0 && cur != device) (void)hipSetDevice(cur);
  }
  DevBuf(const DevBuf &) = delete;
  DevBuf &operator=(const DevBuf &) = delete;
};

struct DevRun {
  uint64_t e0, rows, from, to;  // first entry, rows, endpoints of the first entry
};

// Host-visible words in pinned (fine-grained, coherent) host memory that
// kernels store to: 64-B slots of one slab allocated once per process and
// never freed (a check still in flight may write a slot; a slot is reused
// only after its entry waited for the device, ~CachedPlan).
struct PinnedSlots {
  std::mutex mu;
  char *base = nullptr;
  std::vector<unsigned *> free_slots;
  static constexpr size_t kSlots = 4096;
  unsigned *take(int *rc) {
    std::lock_guard<std::mutex> lk(mu);
    if (!base) {
      void *q = nullptr;
      if (hipHostMalloc(&q, kSlots * 64, hipHostMallocCoherent) != hipSuccess || !q) {
        *rc = set_error(GP_ERR_HIP, "plan cache hipHostMalloc");
        return nullptr;
      }
      base = static_cast<char *>(q);
      for (size_t i = kSlots; i-- > 0;) free_slots.push_back(reinterpret_cast<unsigned *>(base + 64 * i));
    }
    if (free_slots.empty()) {
      *rc = set_error(GP_ERR_HIP, "plan cache: no host-visible slot left");
      return nullptr;
    }
    unsigned *w = free_slots.back();
    free_slots.pop_back();
    *rc = GP_OK;
    return w;
  }
  void give(unsigned *w) {
    std::lock_guard<std::mutex> lk(mu);
    free_slots.push_back(w);
  }
};
PinnedSlots g_pinned_slots;

struct PinnedWord {
  unsigned *p = nullptr;
  int device = 0;
  PinnedWord(int dev, int *rc) : device(dev) {
    p = g_pinned_slots.take(rc);
    if (p) __atomic_store_n(p, 0u, __ATOMIC_RELEASE);
  }
  ~PinnedWord() {
    if (p) g_pinned_slots.give(p);
  }
  unsigned load() const { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }
  PinnedWord(const PinnedWord &) = delete;
  PinnedWord &operator=(const PinnedWord &) = delete;
};

// An entry is immutable once in the cache.  The first call with an index
// leaves a steady-state entry (an inverse map or a ranges plan, with the
// index's compact copy) or, for a scatter of rows over 128 floats, a
// copy-only entry (`sorted` null); the next call with the same content then
// builds the destination-sorted residual into a new entry that shares the
// copy.
struct CachedPlan {
  PlanKey key{};
  std::shared_ptr<DevBuf> copy;    // the index as first seen
  std::shared_ptr<DevBuf> sorted;  // its residual, offsets applied, ascending destination
  // copy-only entry: the buffer its sorted residual will go to, allocated on
  // the first call (the allocation overlaps that call's kernels)
  std::shared_ptr<DevBuf> spare;
  size_t resid = 0;
  std::vector<DevRun> runs;    // with `sorted`: the index's dense runs (the rest is the residual)
  // with `sorted`, the steady state's gate: kGateSlots device words (call
  // generation g uses word g % kGateSlots) then the compact copy's base0 (8
  // B), the host-visible "the index changed" word, and the generation counter
  // (0 never used)
  std::shared_ptr<DevBuf> gate;
  std::shared_ptr<PinnedWord> changed;
  std::atomic<unsigned> gen{0};
  // with `sorted`: the compact copy (id1 as 4 B, index_verify_kernel), whether
  // the index has that shape (host-visible, set by compact_copy_kernel), and
  // what the host knows of it: -1 not yet (the build may still run), 0 no, 1 yes
  std::shared_ptr<DevBuf> compact;
  std::shared_ptr<PinnedWord> compact_broken;
  std::atomic<int> compact_state{-1};
  // an inverse plan (instead of `sorted`): the residual as an inverse map over
  // destination rows 0 .. inv_rows - 1 (inverse_scatter_kernel)
  std::shared_ptr<DevBuf> inv;
  size_t inv_rows = 0;
  // a ranges plan (a gather, or a residual whose destinations ascend): the
  // residual is the call's own index over these entry ranges, in call order
  bool ranges = false;
  bool ascending = false;
  EntryRanges rr{};
  hipEvent_t ready = nullptr;  // recorded once copy (and sorted) are built, on the building stream
  uint64_t last_use = 0;
  size_t bytes = 0;
  const gp_double_index *copy_ptr() const { return static_cast<const gp_double_index *>(copy->p); }
  const gp_double_index *sorted_ptr() const {
    return sorted ? static_cast<const gp_double_index *>(sorted->p) : nullptr;
  }
  bool planned() const { return sorted || inv || ranges; }  // a steady-state entry
  const uint64_t *inv_ptr() const { return static_cast<const uint64_t *>(inv->p); }
  unsigned *gate_words() const { return static_cast<unsigned *>(gate->p); }
  uint64_t *base0_word() const { return reinterpret_cast<uint64_t *>(gate_words() + kGateSlots); }
  // compact_copy_kernel's "not of the compact shape", for the device's kernels
  // (every block of a launch reading the host-visible word costs ~1 ms)
  unsigned *dev_broken_word() const { return reinterpret_cast<unsigned *>(base0_word() + 1); }
  // inverse_count_kernel's listed-row count and finished-wave count
  unsigned long long *count_words() const { return reinterpret_cast<unsigned long long *>(base0_word() + 2); }
  // the inverse map was found unsound at its build (sticky: index_verify_kernel
  // reads it on every later call)
  unsigned *unsound_word() const { return reinterpret_cast<unsigned *>(base0_word() + 4); }
  // The streams this entry's calls ran on, each with an event recorded after
  // the call's last launch (mark_used): what the device may still be doing
  // with the entry's buffers when the host drops it.
  // `unrecorded`: some call's event could not be created or recorded (e.g. a
  // stream of another device than the current one): its launches are not
  // covered by `uses` (a never-recorded event queries as passed), so the drop
  // waits for the device instead.
  std::mutex use_mu;
  std::vector<std::pair<hipStream_t, hipEvent_t>> uses;
  bool unrecorded = false;
  void mark_used(hipStream_t s) {
    std::lock_guard<std::mutex> lk(use_mu);
    hipEvent_t ev = nullptr;
    for (auto &u : uses)
      if (u.first == s) ev = u.second;
    if (!ev) {
      if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
        (void)hipGetLastError();
        unrecorded = true;
        return;
      }
      uses.emplace_back(s, ev);
    }
    if (hipEventRecord(ev, s) != hipSuccess) {
      (void)hipGetLastError();
      unrecorded = true;
    }
  }
  ~CachedPlan();
};

// A dropped or evicted entry's buffers and host-visible words, kept until the
// device has passed every event of its calls (kernels of a call may still read
// or write them): then freed in stream order.  An entry's drop never waits for
// the device -- round 4 synchronised the whole device here, stalling every
// stream of the process, libgeeps' server and reader streams included (ADVICE
// r04).  Reaped at later unplanned calls and cache operations.
struct Grave {
  int device = 0;
  std::vector<hipEvent_t> events;
  hipEvent_t ready = nullptr;
  std::vector<std::shared_ptr<DevBuf>> bufs;
  std::vector<std::shared_ptr<PinnedWord>> words;
};
std::mutex g_graves_mu;
// never destroyed: at process exit the runtime may be gone before static destructors
std::vector<Grave> &g_graves = *new std::vector<Grave>();

void reap_graves() {
  std::vector<Grave> done;
  {
    std::lock_guard<std::mutex> lk(g_graves_mu);
    for (auto it = g_graves.begin(); it != g_graves.end();) {
      bool passed = true;
      for (hipEvent_t e : it->events)
        if (hipEventQuery(e) != hipSuccess) {
          (void)hipGetLastError();  // "not ready" is not a caller's error
          passed = false;
          break;
        }
      if (passed) {
        done.push_back(std::move(*it));
        it = g_graves.erase(it);
      } else {
        ++it;
      }
    }
  }
  for (Grave &g : done) {  // outside the lock: frees (hipFreeAsync) and slot returns
    for (hipEvent_t e : g.events) (void)hipEventDestroy(e);
    if (g.ready) (void)hipEventDestroy(g.ready);
  }
}

CachedPlan::~CachedPlan() {
  if (!ready) return;
  // every call that used the entry already done (the usual case when the
  // host drops it: an idle device): free now, as the member destructors do
  bool passed = !uses.empty() && !unrecorded;
  for (auto &u : uses)
    if (passed && hipEventQuery(u.second) != hipSuccess) {
      (void)hipGetLastError();
      passed = false;
    }
  if (passed) {
    for (auto &u : uses) (void)hipEventDestroy(u.second);
    (void)hipEventDestroy(ready);
    return;
  }
  Grave g;
  g.device = key.device;
  for (auto &u : uses) g.events.push_back(u.second);
  g.ready = ready;
  for (auto *b : {&copy, &sorted, &spare, &gate, &compact, &inv})
    if (*b) g.bufs.push_back(std::move(*b));
  for (auto *w : {&changed, &compact_broken})
    if (*w) g.words.push_back(std::move(*w));
  if (g.events.empty() || unrecorded) {  // launches no event covers (a failed build, a failed record): wait for the device
    int cur = -1;
    (void)hipGetDevice(&cur);
    if (cur != key.device) (void)hipSetDevice(key.device);
    (void)hipDeviceSynchronize();
    if (cur >= 0 && cur != key.device) (void)hipSetDevice(cur);
  }
  std::lock_guard<std::mutex> lk(g_graves_mu);
  g_graves.push_back(std::move(g));
}

// The entries the current unplanned call found or built (cache_find /
// cache_insert on this thread): each gets mark_used on the call's stream once
// the call has issued its last launch.
thread_local std::vector<std::shared_ptr<CachedPlan>> t_touched;

// gp_unplanned_stats_get's counters, in its field order
enum UnplannedStat { kScans, kSteadyCalls, kStaleDrops, kInversePlans, kSortedPlans, kRangesPlans, kNumStats };
std::atomic<uint64_t> g_unplanned_stats[kNumStats];
inline void count_stat(UnplannedStat k) { g_unplanned_stats[k].fetch_add(1, std::memory_order_relaxed); }

std::mutex g_plan_cache_mu;
std::vector<std::shared_ptr<CachedPlan>> g_plan_cache;  // g_plan_cache_mu
uint64_t g_plan_cache_tick = 0;                          // g_plan_cache_mu

std::shared_ptr<CachedPlan> cache_find(const PlanKey &k) {
  std::lock_guard<std::mutex> lk(g_plan_cache_mu);
  for (auto &p : g_plan_cache)
    if (p->key == k) {
      p->last_use = ++g_plan_cache_tick;
      t_touched.push_back(p);
      return p;
    }
  return nullptr;
}

void cache_drop(const std::shared_ptr<CachedPlan> &p) {
  std::lock_guard<std::mutex> lk(g_plan_cache_mu);
  g_plan_cache.erase(std::remove(g_plan_cache.begin(), g_plan_cache.end(), p), g_plan_cache.end());
}

void cache_insert(std::shared_ptr<CachedPlan> p) {
  std::vector<std::shared_ptr<CachedPlan>> evicted;  // freed outside the lock
  {
    std::lock_guard<std::mutex> lk(g_plan_cache_mu);
    for (auto it = g_plan_cache.begin(); it != g_plan_cache.end();)  // a concurrent build of the same key
      if ((*it)->key == p->key) {
        evicted.push_back(*it);
        it = g_plan_cache.erase(it);
      } else {
        ++it;
      }
    p->last_use = ++g_plan_cache_tick;
    t_touched.push_back(p);
    g_plan_cache.push_back(std::move(p));
    auto total = [] {
      size_t b = 0;
      for (auto &q : g_plan_cache) b += q->bytes;
      return b;
    };
    const size_t cap = g_plan_cache_bytes.load(std::memory_order_relaxed);
    // (the newest entry stays even past the cap, unless the cap is 0)
    while (g_plan_cache.size() > (cap ? 1u : 0u) && (g_plan_cache.size() > kPlanCacheEntries || total() > cap)) {
      auto lru = std::min_element(g_plan_cache.begin(), g_plan_cache.end(),
                                  [](const auto &a, const auto &b) { return a->last_use < b->last_use; });
      evicted.push_back(*lru);
      g_plan_cache.erase(lru);
    }
  }
}

// A copy-only entry for an index seen for the first time (its copy, taken on
// stream s after the call's own launches): what the next call's scan compares.
int cache_first_sighting(const PlanKey &key, const gp_double_index *idx, size_t resid, hipStream_t s) {
  auto p = std::make_shared<CachedPlan>();
  p->key = key;
  p->resid = resid;
  p->bytes = (key.n + resid) * sizeof(gp_double_index);
  int rc = GP_OK;
  p->copy = std::make_shared<DevBuf>(key.n * sizeof(gp_double_index), key.device, s, &rc);
  if (rc != GP_OK) return rc;
  p->spare = std::make_shared<DevBuf>(resid * sizeof(gp_double_index), key.device, s, &rc);
  if (rc != GP_OK) return rc;
  GP_HIP_TRY(hipEventCreateWithFlags(&p->ready, hipEventDisableTiming));
  GP_HIP_TRY(hipMemcpyAsync(p->copy->p, idx, key.n * sizeof(gp_double_index), hipMemcpyDeviceToDevice, s));
  GP_HIP_TRY(hipEventRecord(p->ready, s));
  cache_insert(std::move(p));
  return GP_OK;
}

// What a steady-state entry needs besides its plan: the gate words, the
// host-visible "changed" word, and the compact copy of the index (built on s);
// with `copy_if_broken`, also the full copy into p->copy, written only if the
// index is not of the compact shape (else nothing reads it).
int steady_state_setup(CachedPlan *p, const gp_double_index *idx, hipStream_t s, bool copy_if_broken = false) {
  const PlanKey &key = p->key;
  int rc = GP_OK;
  // gate words, base0, broken, the inverse map's two counters, its unsound word
  constexpr size_t kGateBytes = kGateSlots * sizeof(unsigned) + 5 * sizeof(uint64_t);
  p->gate = std::make_shared<DevBuf>(kGateBytes, key.device, s, &rc);
  if (rc != GP_OK) return rc;
  p->changed = std::make_shared<PinnedWord>(key.device, &rc);
  if (rc != GP_OK) return rc;
  p->compact = std::make_shared<DevBuf>(key.n * sizeof(uint32_t), key.device, s, &rc);
  if (rc != GP_OK) return rc;
  p->compact_broken = std::make_shared<PinnedWord>(key.device, &rc);
  if (rc != GP_OK) return rc;
  p->bytes += key.n * sizeof(uint32_t);
  GP_HIP_TRY(hipMemsetAsync(p->gate->p, 0, kGateBytes, s));
  const size_t g = std::max<size_t>(1, std::min((key.n + kBlock - 1) / kBlock, (size_t)num_cus() * 8));
  hipLaunchKernelGGL(compact_copy_kernel, dim3((unsigned)g), dim3(kBlock), 0, s, idx, key.n,
                     static_cast<uint32_t *>(p->compact->p), p->base0_word(), p->compact_broken->p,
                     p->dev_broken_word());
  if (copy_if_broken)
    hipLaunchKernelGGL(copy_if_broken_kernel, dim3((unsigned)g), dim3(kBlock), 0, s, idx, key.n,
                       static_cast<gp_double_index *>(p->copy->p), p->dev_broken_word());
  GP_HIP_TRY(hipGetLastError());
  return GP_OK;
}

// The first call with an index whose residual has no ascending order: the
// inverse plan (for rows of up to 128 floats, destinations below 2^32 and not
// too sparse, kInvSpread).  It keeps the index's compact copy (or full copy)
// for the steady state's check, builds the inverse map of the residual on s
// (fill, scatter, count: generation `*gen` marks it unsound)
// and returns the entry; the caller
// launches the map's rows gated on soundness and the op-order residual gated
// on the opposite.
template <int OP>
int cache_inverse_plan(const PlanKey &key, const gp_double_index *idx, const EntryRanges &rr,
                       const std::vector<DevRun> &runs, size_t inv_rows, hipStream_t s,
                       std::shared_ptr<CachedPlan> *built, unsigned *gen) {
  auto p = std::make_shared<CachedPlan>();
  p->key = key;
  p->resid = rr.pre[rr.count];
  p->runs = runs;
  p->inv_rows = inv_rows;
  p->bytes = key.n * sizeof(gp_double_index) + inv_rows * sizeof(uint64_t);
  int rc = GP_OK;
  p->copy = std::make_shared<DevBuf>(key.n * sizeof(gp_double_index), key.device, s, &rc);
  if (rc != GP_OK) return rc;
  p->inv = std::make_shared<DevBuf>(inv_rows * sizeof(uint64_t), key.device, s, &rc);
  if (rc != GP_OK) return rc;
  rc = steady_state_setup(p.get(), idx, s, /*copy_if_broken=*/true);
  if (rc != GP_OK) return rc;
  GP_HIP_TRY(hipEventCreateWithFlags(&p->ready, hipEventDisableTiming));
  GP_HIP_TRY(hipMemsetAsync(p->inv->p, 0xff, inv_rows * sizeof(uint64_t), s));
  *gen = ++p->gen;
  unsigned *word = p->gate_words() + *gen % kGateSlots;
  const size_t grid = std::max<size_t>(1, std::min((p->resid + kBlock - 1) / kBlock, (size_t)num_cus() * 8));
  uint64_t *inv = static_cast<uint64_t *>(p->inv->p);
  hipLaunchKernelGGL(inverse_scatter_kernel<OP>, dim3((unsigned)grid), dim3(kBlock), 0, s, idx, rr, key.off0,
                     key.off1, inv, word, p->changed->p, *gen, p->unsound_word());
  const size_t cper = (size_t)kBlock * kCountPerThread;
  const size_t cgrid = std::max<size_t>(1, std::min((inv_rows + cper - 1) / cper, (size_t)num_cus()));
  hipLaunchKernelGGL(inverse_count_kernel, dim3((unsigned)cgrid), dim3(kBlock), 0, s, inv, inv_rows,
                     (uint64_t)p->resid, p->count_words(), word, p->changed->p, *gen, p->unsound_word());
  GP_HIP_TRY(hipGetLastError());
  GP_HIP_TRY(hipEventRecord(p->ready, s));
  *built = p;
  count_stat(kInversePlans);
  cache_insert(std::move(p));
  return GP_OK;
}

// A plan that is the call's dense runs and residual ranges (a gather, or a
// residual already in destination order, or too short to sort): kept with a
// copy of the index (and its compact copy) for the steady state.
int cache_ranges_plan(const PlanKey &key, const gp_double_index *idx, const EntryRanges &rr,
                      const std::vector<DevRun> &runs, bool ascending, hipStream_t s) {
  auto p = std::make_shared<CachedPlan>();
  p->key = key;
  p->resid = rr.pre[rr.count];
  p->runs = runs;
  p->ranges = true;
  p->ascending = ascending;
  p->rr = rr;
  p->bytes = key.n * sizeof(gp_double_index);
  int rc = GP_OK;
  p->copy = std::make_shared<DevBuf>(key.n * sizeof(gp_double_index), key.device, s, &rc);
  if (rc != GP_OK) return rc;
  rc = steady_state_setup(p.get(), idx, s, /*copy_if_broken=*/true);
  if (rc != GP_OK) return rc;
  GP_HIP_TRY(hipEventCreateWithFlags(&p->ready, hipEventDisableTiming));
  GP_HIP_TRY(hipEventRecord(p->ready, s));
  count_stat(kRangesPlans);
  cache_insert(std::move(p));
  return GP_OK;
}

// The inverse plan's rows: row_wave_kernel walking destination rows 0 ..
// inv_rows - 1 through the map (Gate::inv), offsets already applied.
template <int OP>
int launch_inverse_rows(float *y, const float *x, const CachedPlan &p, size_t W, size_t limit, hipStream_t s,
                        Gate g) {
  g.inv = p.inv_ptr();
  // (`index` is not read in this form: the map's pointer stands in for it)
  launch_row_op_t<f4, 4, OP, kFlat>(y, x, reinterpret_cast<const gp_double_index *>(p.inv_ptr()), p.inv_rows, 0, 0,
                                    W, limit, SegArg<kFlat>{}, /*sorted=*/true, s, &g);
  GP_HIP_TRY(hipGetLastError());
  return GP_OK;
}

// The second call with the same index: its residual's destination-sorted copy
// (a hipCUB radix sort, gp_sort.hip), built on stream s into a new entry that
// shares `seen`'s copy; returned for this call to run.
template <int OP>
int cache_second_sighting(const std::shared_ptr<CachedPlan> &seen, const gp_double_index *idx,
                          const EntryRanges &rr, const std::vector<DevRun> &runs, uint64_t max_dst,
                          hipStream_t s, std::shared_ptr<CachedPlan> *built) {
  const PlanKey &key = seen->key;
  const size_t resid = rr.pre[rr.count];
  auto p = std::make_shared<CachedPlan>();
  p->key = key;
  p->resid = resid;
  p->runs = runs;
  p->bytes = (key.n + resid) * sizeof(gp_double_index);
  p->copy = seen->copy;
  int rc = GP_OK;
  if (seen->spare)
    p->sorted = seen->spare;  // written only here: no call reads a copy-only entry's spare
  else
    p->sorted = std::make_shared<DevBuf>(resid * sizeof(gp_double_index), key.device, s, &rc);
  if (rc != GP_OK) return rc;
  rc = steady_state_setup(p.get(), idx, s);
  if (rc != GP_OK) return rc;
  GP_HIP_TRY(hipEventCreateWithFlags(&p->ready, hipEventDisableTiming));
  uint32_t *kv = nullptr;  // keys, values, sorted keys, sorted values
  GP_HIP_TRY(hipMallocAsync(reinterpret_cast<void **>(&kv), 4 * resid * sizeof(uint32_t), s));
  const size_t grid = std::min((resid + kBlock - 1) / kBlock, (size_t)num_cus() * 8);
  hipLaunchKernelGGL(residual_keys_kernel<OP>, dim3((unsigned)grid), dim3(kBlock), 0, s, idx, rr, key.off0, key.off1,
                     kv, kv + resid);
  int end_bit = 1;  // destination rows are below 2^32 here (checked by the caller)
  while (end_bit < 32 && (max_dst >> end_bit)) ++end_bit;
  rc = radix_sort_pairs_u32(kv, kv + 2 * resid, kv + resid, kv + 3 * resid, resid, end_bit, s);
  if (rc == GP_OK) {
    hipLaunchKernelGGL(residual_gather_kernel<OP>, dim3((unsigned)grid), dim3(kBlock), 0, s, idx, kv + 3 * resid,
                       resid, key.off0, key.off1, static_cast<gp_double_index *>(p->sorted->p));
    rc = hipGetLastError() == hipSuccess ? GP_OK : set_error(GP_ERR_HIP, "residual_gather_kernel launch");
  }
  GP_HIP_TRY(hipFreeAsync(kv, s));
  if (rc != GP_OK) return rc;
  GP_HIP_TRY(hipEventRecord(p->ready, s));
  *built = p;
  count_stat(kSortedPlans);
  cache_insert(std::move(p));
  return GP_OK;
}

// The analysed form of launch_row_op (see the section comment).
template <int OP>
int launch_row_op_analyzed_body(float *y, const float *x, const gp_double_index *idx, size_t n, gp_double_index off,
                                size_t row_size, size_t limit, hipStream_t s);
template <int OP>
int launch_row_op_analyzed(float *y, const float *x, const gp_double_index *idx, size_t n, gp_double_index off,
                           size_t row_size, size_t limit, hipStream_t s) {
  reap_graves();
  t_touched.clear();
  const int rc = launch_row_op_analyzed_body<OP>(y, x, idx, n, off, row_size, limit, s);
  for (auto &p : t_touched) p->mark_used(s);  // after the call's last launch
  t_touched.clear();
  return rc;
}
template <int OP>
int launch_row_op_analyzed_body(float *y, const float *x, const gp_double_index *idx, size_t n, gp_double_index off,
                                size_t row_size, size_t limit, hipStream_t s) {
  const size_t W = row_size;
  const size_t tiles = (n + 63) / 64, groups = (tiles + kScanGroupTiles - 1) / kScanGroupTiles;
  keep_pool_memory();
  int dev = 0;
  GP_HIP_TRY(hipGetDevice(&dev));
  const PlanKey key{dev, OP, reinterpret_cast<uintptr_t>(idx), n, W, limit, off.id0, off.id1};
  std::shared_ptr<CachedPlan> cached = cache_find(key);
  // a steady-state call since the last host look found the index changed: the
  // entry is stale, plan this call afresh (scan, host round trip)
  if (cached && cached->planned() && cached->changed->load() != 0) {
    count_stat(kStaleDrops);
    cache_drop(cached);
    cached.reset();
  }
  // its copy (and sorted residual) may still be in flight on the stream that built them
  if (cached) GP_HIP_TRY(hipStreamWaitEvent(s, cached->ready, 0));
  auto launch_runs = [&](const std::vector<DevRun> &rs, const Gate *g) {
    for (const DevRun &r : rs) {
      BucketPtrs b = {};
      b.p[0] = x + r.from * W;
      float *yr = y + r.to * W;
      int rc;
      if constexpr (OP == kAddFrom)
        rc = launch_bucket_sum_nb<1>(yr, yr, b, r.rows * W, s, g);
      else if constexpr (OP == kInitFrom)
        rc = launch_bucket_sum_nb<1, true>(yr, nullptr, b, r.rows * W, s, g);
      else
        rc = launch_bucket_sum_nb<0>(yr, x + r.from * W, BucketPtrs{}, r.rows * W, s, g);
      if (rc != GP_OK) return rc;
    }
    return (int)GP_OK;
  };
  if (cached && cached->planned()) {
    // The steady state: a planned index seen again.  Check it against the copy
    // and launch both outcomes behind the check, each gated on its result:
    // the cached dense runs and sorted residual (unchanged), or this call's
    // rows in op order (changed; as a first call runs its residual).  Exactly
    // one does any work; nothing waits for the host.
    count_stat(kSteadyCalls);
    unsigned gen = ++cached->gen;
    if (gen == 0) gen = ++cached->gen;  // 0 is the gate words' initial value
    unsigned *word = cached->gate_words() + gen % kGateSlots;
    // the check's form once the host knows the compact copy's build finished
    // (never waits); until then the device reads the build's flag (FORM 2)
    int compact = cached->compact_state.load(std::memory_order_acquire);
    if (compact < 0) {
      const hipError_t q = hipEventQuery(cached->ready);
      if (q == hipSuccess) {
        compact = cached->compact_broken->load() ? 0 : 1;
        cached->compact_state.store(compact, std::memory_order_release);
      } else {
        (void)hipGetLastError();  // "not ready" is not this call's error
      }
    }
    const size_t per_block = (size_t)kBlock * kCmpPerThread;
    const size_t grid = std::max<size_t>(1, std::min((n + per_block - 1) / per_block, (size_t)num_cus() * 8));
    auto verify = compact == 1   ? &index_verify_kernel<1>
                  : compact == 0 ? &index_verify_kernel<0>
                                 : &index_verify_kernel<2>;
    hipLaunchKernelGGL(verify, dim3((unsigned)grid), dim3(kBlock), 0, s, idx, cached->copy_ptr(),
                       static_cast<const uint32_t *>(cached->compact->p), n, cached->base0_word(), word,
                       cached->changed->p, gen, cached->dev_broken_word(), cached->unsound_word());
    GP_HIP_TRY(hipGetLastError());
    // dense runs only if unchanged; one row launch for both outcomes: the
    // sorted residual if unchanged, else every row of the call in op order
    const Gate same{word, gen, kGateIfSame, nullptr, 0, 0, 0, nullptr};
    const Gate select{word, gen, kGateSelect, idx, n, off.id0, off.id1, nullptr};
    int rc = launch_runs(cached->runs, &same);
    if (rc != GP_OK) return rc;
    if (cached->inv) return launch_inverse_rows<OP>(y, x, *cached, W, limit, s, select);
    if (cached->ranges) {
      // the residual is the call's own index over the kept ranges, in call
      // order: the first range's launch selects (all the call's rows if the
      // index changed), the others run only if it did not; with no residual,
      // the op-order form alone, gated on a change
      const EntryRanges &rr = cached->rr;
      if (rr.count == 0) {
        const Gate changed{word, gen, kGateIfChanged, nullptr, 0, 0, 0, nullptr};
        return launch_row_op<OP>(y, x, idx, n, off, W, limit, s, /*sorted=*/false, &changed);
      }
      for (uint32_t i = 0; i < rr.count; ++i) {
        rc = launch_row_op<OP>(y, x, idx + rr.lo[i], rr.hi[i] - rr.lo[i], off, W, limit, s, cached->ascending,
                               i == 0 ? &select : &same);
        if (rc != GP_OK) return rc;
      }
      return GP_OK;
    }
    return launch_row_op<OP>(y, x, cached->sorted_ptr(), cached->resid, gp_double_index{0, 0}, W, limit, s,
                             /*sorted=*/true, &select);
  }
  count_stat(kScans);
  const size_t scan_bytes = kScanWordsOff + groups * kScanWords * sizeof(uint64_t);
  char *ws = nullptr;
  GP_HIP_TRY(hipMallocAsync(reinterpret_cast<void **>(&ws), scan_bytes, s));
  struct Free {  // the workspace goes back in stream order, whatever happens
    char *&p;
    hipStream_t s;
    ~Free() {
      if (p) (void)hipFreeAsync(p, s);
    }
  } free_ws{ws, s};
  GP_HIP_TRY(hipMemsetAsync(ws, 0, sizeof(ScanHeader), s));
  {
    const size_t grid = std::max<size_t>(1, std::min(groups, (size_t)num_cus() * 8));
    if (cached)
      hipLaunchKernelGGL((index_scan_kernel<OP, true>), dim3((unsigned)grid), dim3(kBlock), 0, s, idx, n, off.id0,
                         off.id1, W, limit, cached->copy_ptr(), ws);
    else
      hipLaunchKernelGGL((index_scan_kernel<OP, false>), dim3((unsigned)grid), dim3(kBlock), 0, s, idx, n, off.id0,
                         off.id1, W, limit, nullptr, ws);
    GP_HIP_TRY(hipGetLastError());
  }
  char *h = static_cast<char *>(g_scan_landing.get(scan_bytes));
  if (!h) return set_error(GP_ERR_HIP, "pinned scan buffer");
  GP_HIP_TRY(hipMemcpyAsync(h, ws, scan_bytes, hipMemcpyDeviceToHost, s));
  GP_HIP_TRY(hipStreamSynchronize(s));
  const ScanHeader hdr = *reinterpret_cast<const ScanHeader *>(h);
  const RunStart *st = reinterpret_cast<const RunStart *>(h + sizeof(ScanHeader));
  const uint64_t *words = reinterpret_cast<const uint64_t *>(h + kScanWordsOff);
  auto bit = [&](size_t t, int w) {
    return (words[kScanWords * (t / kScanGroupTiles) + w] >> (t % kScanGroupTiles)) & 1;
  };
  uint64_t max_dst = 0;
  for (size_t g = 0; g < groups; ++g) max_dst = std::max(max_dst, words[kScanWords * g + 3]);
  if (cached && hdr.mismatches) {  // the same pointer now holds another index
    cache_drop(cached);
    cached.reset();
  }

  // dense runs at tile granularity, long enough for the sweep forms, whose
  // first entry the scan recorded; the longest kMaxDeviceRuns of them
  const size_t min_tiles = std::max<size_t>(1, kDenseRunBytes / (64 * W * sizeof(float)));
  std::vector<DevRun> runs;
  {
    const unsigned ns = std::min<unsigned>(hdr.n_starts, kMaxRunStarts);
    std::vector<RunStart> starts(st, st + ns);
    std::sort(starts.begin(), starts.end(), [](const RunStart &a, const RunStart &b) { return a.tile < b.tile; });
    // first tile >= t that is not dense-and-continuing (word at a time)
    auto run_end = [&](size_t t) {
      while (t < tiles) {
        const size_t g = t / kScanGroupTiles;
        const uint64_t brk = ~(words[kScanWords * g] & words[kScanWords * g + 1]) >> (t % kScanGroupTiles);
        if (brk) return std::min(tiles, t + (size_t)__builtin_ctzll(brk));
        t = (g + 1) * kScanGroupTiles;
      }
      return tiles;
    };
    for (const RunStart &r : starts) {
      const size_t t = run_end(r.tile + 1);
      if (t - r.tile >= min_tiles) {
        const uint64_t e0 = r.tile * 64, rows = std::min<uint64_t>((t - r.tile) * 64, n - e0);
        runs.push_back(DevRun{e0, rows, r.from, r.to});
      }
    }
    if (runs.size() > (size_t)kMaxDeviceRuns) {
      std::nth_element(runs.begin(), runs.begin() + kMaxDeviceRuns, runs.end(),
                       [](const DevRun &a, const DevRun &b) { return a.rows > b.rows; });
      runs.resize(kMaxDeviceRuns);
      std::sort(runs.begin(), runs.end(), [](const DevRun &a, const DevRun &b) { return a.e0 < b.e0; });
    }
  }
  if (const int rc = launch_runs(runs, nullptr); rc != GP_OK) return rc;
  // the residual: entry ranges between the runs
  EntryRanges rr = {};
  {
    uint64_t at = 0;
    auto add = [&](uint64_t lo, uint64_t hi) {
      if (hi <= lo) return;
      rr.lo[rr.count] = lo;
      rr.hi[rr.count] = hi;
      rr.pre[rr.count + 1] = rr.pre[rr.count] + (hi - lo);
      ++rr.count;
    };
    for (const DevRun &r : runs) {
      add(at, r.e0);
      at = r.e0 + r.rows;
    }
    add(at, n);
  }
  const size_t resid = rr.pre[rr.count];
  if (resid == 0) return cached ? GP_OK : cache_ranges_plan(key, idx, rr, runs, true, s);  // all dense runs
  // destinations already (mostly) ascending: the call's order is the sorted one
  size_t resid_tiles = 0, asc_tiles = 0;
  for (uint32_t i = 0; i < rr.count; ++i) {
    size_t t = rr.lo[i] / 64;
    const size_t t1 = (rr.hi[i] + 63) / 64;
    resid_tiles += t1 - t;
    for (; t < t1 && t % kScanGroupTiles; ++t) asc_tiles += bit(t, 2);
    for (; t + kScanGroupTiles <= t1; t += kScanGroupTiles)
      asc_tiles += __builtin_popcountll(words[kScanWords * (t / kScanGroupTiles) + 2]);
    for (; t < t1; ++t) asc_tiles += bit(t, 2);
  }
  const bool ascending = asc_tiles * 10 >= resid_tiles * 9;
  // a scatter's large unsorted residual is worth a destination-sorted copy
  // when the index comes back: the second call with the same content builds
  // it (one radix sort, about what sorting saves in one call) and runs it
  const bool sortable = OP != kAssignTo && !ascending && resid * W * sizeof(float) >= kSortMinBytes &&
                        max_dst < (1ull << 32) && n < (1ull << 32);
  // the inverse plan: rows of up to 128 floats (the wave kernel's shapes),
  // destinations not too sparse for a map over 0 .. max_dst
  const size_t inv_rows = (size_t)max_dst + 1;
  const bool inverse = sortable && !cached && W / 4 <= 32 && inv_rows <= kInvSpread * resid + (1u << 20);
  if (inverse) {
    std::shared_ptr<CachedPlan> built;
    unsigned gen = 0;
    int rc = cache_inverse_plan<OP>(key, idx, rr, runs, inv_rows, s, &built, &gen);
    if (rc != GP_OK) return rc;
    unsigned *word = built->gate_words() + gen % kGateSlots;
    // the map's rows if it is sound, else the residual in op order (as the
    // calls before ABI 11 ran it)
    rc = launch_inverse_rows<OP>(y, x, *built, W, limit, s, Gate{word, gen, kGateIfSame, nullptr, 0, 0, 0, nullptr});
    if (rc != GP_OK) return rc;
    const Gate unsound{word, gen, kGateIfChanged, nullptr, 0, 0, 0, nullptr};
    for (uint32_t i = 0; i < rr.count; ++i) {
      rc = launch_row_op<OP>(y, x, idx + rr.lo[i], rr.hi[i] - rr.lo[i], off, W, limit, s, ascending, &unsound);
      if (rc != GP_OK) return rc;
    }
    return GP_OK;
  }
  if (sortable && cached && !cached->sorted && cached->resid == resid) {
    std::shared_ptr<CachedPlan> built;
    const int rc = cache_second_sighting<OP>(cached, idx, rr, runs, max_dst, s, &built);
    if (rc != GP_OK) return rc;
    return launch_row_op<OP>(y, x, built->sorted_ptr(), resid, gp_double_index{0, 0}, W, limit, s,
                             /*sorted=*/true);
  }
  for (uint32_t i = 0; i < rr.count; ++i) {
    const int rc = launch_row_op<OP>(y, x, idx + rr.lo[i], rr.hi[i] - rr.lo[i], off, W, limit, s, ascending);
    if (rc != GP_OK) return rc;
  }
  // first sighting: remember the content, so the next call can tell it is the same
  if (sortable && !cached) return cache_first_sighting(key, idx, resid, s);
  // nothing to sort (a gather, ascending destinations, a short residual): the
  // plan is the runs and the residual ranges themselves, kept for the steady
  // state's check-and-run without a scan
  if (!sortable && !cached) return cache_ranges_plan(key, idx, rr, runs, ascending, s);
  return GP_OK;
}

// The unplanned calls: large ones plan themselves on the device.
template <int OP>
int launch_row_op_unplanned(float *y, const float *x, const gp_double_index *idx, size_t n, gp_double_index off,
                            size_t row_size, size_t limit, hipStream_t s) {
  if (n == 0) return GP_OK;
  if (!y || !x || !idx) return set_error(GP_ERR_INVALID, "null pointer");
  if (row_size == 0) return set_error(GP_ERR_INVALID, "row_size == 0");
  const size_t min_bytes = g_analyze_min_bytes.load(std::memory_order_relaxed);
  if (min_bytes != SIZE_MAX && n * row_size * sizeof(float) >= min_bytes && row_size % 4 == 0 && aligned16(y) &&
      aligned16(x))
    return launch_row_op_analyzed<OP>(y, x, idx, n, off, row_size, limit, s);
  return launch_row_op<OP>(y, x, idx, n, off, row_size, limit, s);
}

int create_plan(gp_row_plan *plan, const gp_double_index *host_index, size_t num_rows,
                gp_double_index offset, size_t row_size, size_t num_vals_limit, bool gather);

}  // namespace

// ===========================================================================
// C-ABI
// ===========================================================================
extern "C" {

int gp_abi_version(void) { return GP_ABI_VERSION; }

int gp_set_unplanned_min_bytes(size_t min_bytes) {
  g_analyze_min_bytes.store(min_bytes, std::memory_order_relaxed);
  return GP_OK;
}

int gp_unplanned_cache_clear(void) {
  {
    std::vector<std::shared_ptr<CachedPlan>> gone;  // freed outside the lock
    std::lock_guard<std::mutex> lk(g_plan_cache_mu);
    gone.swap(g_plan_cache);
  }
  reap_graves();
  return GP_OK;
}

int gp_unplanned_stats_get(gp_unplanned_stats *out) {
  if (!out) return set_error(GP_ERR_INVALID, "null pointer");
  uint64_t *f[kNumStats] = {&out->scans,         &out->steady_calls, &out->stale_drops,
                            &out->inverse_plans, &out->sorted_plans, &out->ranges_plans};
  for (int k = 0; k < kNumStats; ++k) *f[k] = g_unplanned_stats[k].load(std::memory_order_relaxed);
  return GP_OK;
}

int gp_unplanned_cache_entries(size_t *entries, size_t *bytes) {
  if (!entries || !bytes) return set_error(GP_ERR_INVALID, "null pointer");
  std::lock_guard<std::mutex> lk(g_plan_cache_mu);
  *entries = g_plan_cache.size();
  *bytes = 0;
  for (auto &p : g_plan_cache) *bytes += p->bytes;
  return GP_OK;
}

int gp_set_unplanned_cache_bytes(size_t max_bytes) {
  reap_graves();
  g_plan_cache_bytes.store(max_bytes, std::memory_order_relaxed);
  std::vector<std::shared_ptr<CachedPlan>> evicted;  // freed outside the lock
  {
    std::lock_guard<std::mutex> lk(g_plan_cache_mu);
    size_t total = 0;
    for (auto &p : g_plan_cache) total += p->bytes;
    while (!g_plan_cache.empty() && total > max_bytes) {
      auto lru = std::min_element(g_plan_cache.begin(), g_plan_cache.end(),
                                  [](const auto &a, const auto &b) { return a->last_use < b->last_use; });
      total -= (*lru)->bytes;
      evicted.push_back(*lru);
      g_plan_cache.erase(lru);
    }
  }
  return GP_OK;
}

const char *gp_last_error(void) { return g_last_error.c_str(); }

int gp_scatter_add_rows(float *y, const float *x, const gp_double_index *index,
                        size_t num_rows, gp_double_index offset,
                        size_t row_size, size_t num_vals_limit, gp_stream s) {
  return launch_row_op_unplanned<kAddFrom>(y, x, index, num_rows, offset, row_size,
                                 num_vals_limit, (hipStream_t)s);
}

int gp_gather_rows(float *y, const float *x, const gp_double_index *index,
                   size_t num_rows, gp_double_index offset, size_t row_size,
                   size_t num_vals_limit, gp_stream s) {
  return launch_row_op_unplanned<kAssignTo>(y, x, index, num_rows, offset, row_size,
                                  num_vals_limit, (hipStream_t)s);
}

int gp_scatter_rows(float *y, const float *x, const gp_double_index *index,
                    size_t num_rows, gp_double_index offset, size_t row_size,
                    size_t num_vals_limit, gp_stream s) {
  return launch_row_op<kAssignFrom>(y, x, index, num_rows, offset, row_size,
                                    num_vals_limit, (hipStream_t)s);
}

int gp_scatter_init_rows(float *y, const float *x, const gp_double_index *index,
                         size_t num_rows, gp_double_index offset, size_t row_size,
                         size_t num_vals_limit, gp_stream s) {
  return launch_row_op_unplanned<kInitFrom>(y, x, index, num_rows, offset, row_size,
                                  num_vals_limit, (hipStream_t)s);
}

int gp_gather_rows_segmented(float *y, const gp_row_segments *x_segments,
                             const gp_double_index *index, size_t num_rows,
                             gp_double_index offset, size_t row_size,
                             size_t num_vals_limit, gp_stream s) {
  return launch_row_op_seg<kAssignTo, kSegX>(y, x_segments, index, num_rows, offset, row_size,
                                             num_vals_limit, (hipStream_t)s);
}

int gp_scatter_add_rows_segmented(const gp_row_segments *y_segments, const float *x,
                                  const gp_double_index *index, size_t num_rows,
                                  gp_double_index offset, size_t row_size,
                                  size_t num_vals_limit, gp_stream s) {
  return launch_row_op_seg<kAddFrom, kSegY>(const_cast<float *>(x), y_segments, index, num_rows,
                                            offset, row_size, num_vals_limit, (hipStream_t)s);
}

int gp_row_plan_create(gp_row_plan *plan, const gp_double_index *host_index, size_t num_rows,
                       gp_double_index offset, size_t row_size, size_t num_vals_limit) {
  return create_plan(plan, host_index, num_rows, offset, row_size, num_vals_limit, false);
}

int gp_gather_plan_create(gp_row_plan *plan, const gp_double_index *host_index, size_t num_rows,
                          gp_double_index offset, size_t row_size, size_t num_vals_limit) {
  return create_plan(plan, host_index, num_rows, offset, row_size, num_vals_limit, true);
}

int gp_gather_rows_planned(float *y, const float *x, gp_row_plan plan, gp_stream s) {
  if (!y || !x) return set_error(GP_ERR_INVALID, "null pointer");
  return launch_gather_planned(y, x, nullptr, plan, (hipStream_t)s);
}

int gp_gather_rows_segmented_planned(float *y, const gp_row_segments *x_segments, gp_row_plan plan,
                                     gp_stream s) {
  if (!y || !x_segments) return set_error(GP_ERR_INVALID, "null pointer");
  return launch_gather_planned(y, nullptr, x_segments, plan, (hipStream_t)s);
}

}  // extern "C"

namespace {
int create_plan(gp_row_plan *plan, const gp_double_index *host_index, size_t num_rows,
                gp_double_index offset, size_t row_size, size_t num_vals_limit, bool gather) {
  if (!plan) return set_error(GP_ERR_INVALID, "null pointer");
  *plan = nullptr;
  if (num_rows && !host_index) return set_error(GP_ERR_INVALID, "null index");
  if (row_size == 0) return set_error(GP_ERR_INVALID, "row_size == 0");
  auto *p = new gp_row_plan_s;
  p->num_rows = num_rows;
  p->row_size = row_size;
  p->limit = num_vals_limit;
  p->gather = gather;
  if (hipGetDevice(&p->device) != hipSuccess) p->device = 0;
  const int rc = build_row_plan(p, host_index, num_rows, offset);
  if (rc != GP_OK) {
    gp_row_plan_destroy(p);
    return rc;
  }
  *plan = p;
  return GP_OK;
}
}  // namespace

extern "C" {

int gp_row_plan_destroy(gp_row_plan plan) {
  if (!plan) return GP_OK;
  hipError_t e = plan->residual ? hipFree(plan->residual) : hipSuccess;
  for (const auto &l : plan->repeats) {
    const hipError_t e2 = hipFree(l.index);
    if (e == hipSuccess) e = e2;
  }
  delete plan;
  GP_HIP_TRY(e);
  return GP_OK;
}

int gp_row_plan_repeats(gp_row_plan plan, size_t *layers, size_t *repeat_rows) {
  if (!plan || !layers || !repeat_rows) return set_error(GP_ERR_INVALID, "null pointer");
  *layers = plan->repeats.size();
  *repeat_rows = plan->repeat_rows;
  return GP_OK;
}

int gp_row_plan_info(gp_row_plan plan, size_t *num_rows, size_t *dense_runs, size_t *dense_rows) {
  if (!plan || !num_rows || !dense_runs || !dense_rows)
    return set_error(GP_ERR_INVALID, "null pointer");
  *num_rows = plan->num_rows;
  *dense_runs = plan->dense.size();
  *dense_rows = plan->dense_rows;
  return GP_OK;
}

int gp_row_plan_launches(gp_row_plan plan, int init, int *sweep_launches, int *phased_launches,
                         int *other_launches) {
  if (!plan || !sweep_launches || !phased_launches || !other_launches)
    return set_error(GP_ERR_INVALID, "null pointer");
  size_t sw = 0, ph = 0, ot = (plan->residual_rows ? 1 : 0) + plan->repeats.size();
  for (const RowRun &r : plan->dense) {
    const size_t n = r.rows * plan->row_size;
    const SumLaunches l = plan->gather ? sum_launches<0>(n)
                          : init       ? sum_launches<1, true>(n)
                                       : sum_launches<1>(n);
    sw += l.sweep + l.sweep_small;
    ph += l.phased;
    ot += l.other;
  }
  *sweep_launches = (int)sw;
  *phased_launches = (int)ph;
  *other_launches = (int)ot;
  return GP_OK;
}

int gp_scatter_add_rows_planned(float *y, const float *x, gp_row_plan plan, gp_stream s) {
  if (!y || !x) return set_error(GP_ERR_INVALID, "null pointer");
  return launch_planned<kAddFrom>(y, x, plan, (hipStream_t)s);
}

int gp_scatter_init_rows_planned(float *y, const float *x, gp_row_plan plan, gp_stream s) {
  if (!y || !x) return set_error(GP_ERR_INVALID, "null pointer");
  return launch_planned<kInitFrom>(y, x, plan, (hipStream_t)s);
}

int gp_bucket_sum_sweep_plan(size_t num_vals, int num_buckets, int *phased_launches,
                             int *reg_tiles, int *sweep_launches) {
  if (!phased_launches || !reg_tiles || !sweep_launches)
    return set_error(GP_ERR_INVALID, "null pointer");
  int *l = phased_launches, *r = reg_tiles, *w = sweep_launches;
  switch (num_buckets) {
    case 1: bucket_sum_plan_nb<1>(num_vals, l, r, w); break;
    case 2: bucket_sum_plan_nb<2>(num_vals, l, r, w); break;
    case 3: bucket_sum_plan_nb<3>(num_vals, l, r, w); break;
    case 4: bucket_sum_plan_nb<4>(num_vals, l, r, w); break;
    case 5: bucket_sum_plan_nb<5>(num_vals, l, r, w); break;
    case 6: bucket_sum_plan_nb<6>(num_vals, l, r, w); break;
    case 7: bucket_sum_plan_nb<7>(num_vals, l, r, w); break;
    case 8: bucket_sum_plan_nb<8>(num_vals, l, r, w); break;
    default: return set_error(GP_ERR_INVALID, "bucket count out of range");
  }
  return GP_OK;
}

int gp_bucket_sum_launch_plan(size_t num_vals, int num_buckets, gp_sum_plan *plan) {
  if (!plan) return set_error(GP_ERR_INVALID, "null pointer");
  switch (num_buckets) {
    case 1: sum_plan_nb<1>(num_vals, plan); break;
    case 2: sum_plan_nb<2>(num_vals, plan); break;
    case 3: sum_plan_nb<3>(num_vals, plan); break;
    case 4: sum_plan_nb<4>(num_vals, plan); break;
    case 5: sum_plan_nb<5>(num_vals, plan); break;
    case 6: sum_plan_nb<6>(num_vals, plan); break;
    case 7: sum_plan_nb<7>(num_vals, plan); break;
    case 8: sum_plan_nb<8>(num_vals, plan); break;
    default: return set_error(GP_ERR_INVALID, "bucket count out of range");
  }
  return GP_OK;
}

int gp_bucket_sum_plan(size_t num_vals, int num_buckets, int *phased_launches,
                       int *reg_tiles) {
  int sweeps = 0;
  return gp_bucket_sum_sweep_plan(num_vals, num_buckets, phased_launches, reg_tiles, &sweeps);
}

int gp_bucket_sum_apply(float *master, const float *const *buckets,
                        int num_buckets, size_t num_vals, gp_stream s) {
  if (num_buckets == 0 || num_vals == 0) return GP_OK;
  if (num_buckets < 0) return set_error(GP_ERR_INVALID, "num_buckets < 0");
  if (!master || !buckets) return set_error(GP_ERR_INVALID, "null pointer");
  for (int k = 0; k < num_buckets; ++k)
    if (!buckets[k]) return set_error(GP_ERR_INVALID, "null bucket pointer");
  // More than kMaxBucketsPerLaunch buckets: consecutive launches over the
  // same master, each continuing the bucket order where the last stopped.
  for (int k0 = 0; k0 < num_buckets; k0 += kMaxBucketsPerLaunch) {
    const int nb = num_buckets - k0 < kMaxBucketsPerLaunch
                       ? num_buckets - k0
                       : kMaxBucketsPerLaunch;
    const int rc = launch_bucket_sum(master, master, buckets + k0, nb,
                                     num_vals, (hipStream_t)s);
    if (rc != GP_OK) return rc;
  }
  return GP_OK;
}

int gp_bucket_sum_into(float *out, const float *in, const float *const *buckets,
                       int num_buckets, size_t num_vals, gp_stream s) {
  if (num_vals == 0) return GP_OK;
  if (num_buckets < 0) return set_error(GP_ERR_INVALID, "num_buckets < 0");
  if (!out || !in || (num_buckets && !buckets)) return set_error(GP_ERR_INVALID, "null pointer");
  if (out != in && out < in + num_vals && in < out + num_vals)
    return set_error(GP_ERR_INVALID, "out and in overlap");
  for (int k = 0; k < num_buckets; ++k)
    if (!buckets[k]) return set_error(GP_ERR_INVALID, "null bucket pointer");
  if (num_buckets == 0) {
    // the copy through the sweep kernels' copy form: an IPC-mapped `in` (a
    // peer process's master version) sends hipMemcpyAsync to a copy engine,
    // measured at 1.3 TB/s for 2 GiB where this runs at the HBM copy rate
    if (out != in) {
      const int rc = launch_bucket_sum_nb<0>(out, in, BucketPtrs{}, num_vals, (hipStream_t)s);
      if (rc != GP_OK) return rc;
      GP_HIP_TRY(hipGetLastError());
    }
    return GP_OK;
  }
  // The first launch reads `in` and writes `out`; any further launches (more
  // than kMaxBucketsPerLaunch buckets) continue in place on `out`.
  const float *src = in;
  for (int k0 = 0; k0 < num_buckets; k0 += kMaxBucketsPerLaunch) {
    const int nb = num_buckets - k0 < kMaxBucketsPerLaunch ? num_buckets - k0
                                                           : kMaxBucketsPerLaunch;
    const int rc = launch_bucket_sum(out, src, buckets + k0, nb, num_vals, (hipStream_t)s);
    if (rc != GP_OK) return rc;
    src = out;
  }
  return GP_OK;
}

int gp_add(size_t n, const float *a, const float *b, float *y, gp_stream s) {
  if (n == 0) return GP_OK;
  if (!a || !b || !y) return set_error(GP_ERR_INVALID, "null pointer");
  const float *bk[1] = {b};
  return launch_bucket_sum(y, a, bk, 1, n, (hipStream_t)s);
}

int gp_hbm_probe(int kind, float *buffer, size_t num_vals, gp_stream s) {
  if (num_vals == 0) return GP_OK;
  if (!buffer || !aligned16(buffer)) return set_error(GP_ERR_INVALID, "null or unaligned buffer");
  if (kind == GP_PROBE_READ) {
    // the buffer is only read (the kernel's sink is a device global of its own)
    const size_t grid = (size_t)num_cus() * 2;
    hipLaunchKernelGGL(hbm_read_probe_kernel, dim3((unsigned)grid), dim3(kBlock), 0, (hipStream_t)s,
                       reinterpret_cast<const f4 *>(buffer), num_vals / 4);
  } else if (kind == GP_PROBE_WRITE) {
    // the runtime's fill kernel: 6.3-6.7 TB/s, above every store-loop shape
    // tried (5.5-6.3 TB/s; profiles/r02/tune/probe_tune*.txt)
    GP_HIP_TRY(hipMemsetAsync(buffer, 0, num_vals * sizeof(float), (hipStream_t)s));
  } else {
    return set_error(GP_ERR_INVALID, "probe kind");
  }
  GP_HIP_TRY(hipGetLastError());
  return GP_OK;
}

int gp_zero(float *y, size_t num_vals, gp_stream s) {
  if (num_vals == 0) return GP_OK;
  if (!y) return set_error(GP_ERR_INVALID, "null pointer");
  GP_HIP_TRY(hipMemsetAsync(y, 0, num_vals * sizeof(float), (hipStream_t)s));
  return GP_OK;
}


}  // extern "C"

// The thread's gp_last_error message, for the C-ABI functions of the library's
// other translation units (gp_host.cpp: host-memory row ops; gp_runtime.hip:
// memory, streams, events, IPC).
namespace gp_internal {
int set_error(int code, const char *msg) { return ::set_error(code, msg); }
}  // namespace gp_internal
