// gp_unplanned.hip — the unplanned row calls of the C-ABI (gp_scatter_add_rows,
// gp_scatter_init_rows, gp_gather_rows: the reference binding's
// add_rows_from_double_index_gpu / assign_rows_to_double_index_gpu, which pass
// a device DoubleIndex on every call, row-op-util.cu:127-142) and the device
// planning behind them: the index scan, the inverse map / sorted residual /
// ranges plans, the plan cache and its gated, host-sync-free steady state
// (DESIGN.md §5.3).  The kernels they launch besides their own come from
// gp_kernels.hpp; the radix sort from gp_sort.hip.

#include "gp_kernels.hpp"

// gp_sort.hip (hipCUB's radix sort, in its own translation unit): sort n
// (key, value) pairs by the low end_bit bits of the key, stream-ordered, on
// temporary storage from the stream-ordered pool.  Returns a GP_* status.
int gp_internal_radix_sort_pairs_u32(const uint32_t *keys_in, uint32_t *keys_out, const uint32_t *vals_in,
                                     uint32_t *vals_out, size_t n, int end_bit, hipStream_t s,
                                     std::string *error);

namespace {

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

}  // namespace

extern "C" {

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

int gp_scatter_init_rows(float *y, const float *x, const gp_double_index *index,
                         size_t num_rows, gp_double_index offset, size_t row_size,
                         size_t num_vals_limit, gp_stream s) {
  return launch_row_op_unplanned<kInitFrom>(y, x, index, num_rows, offset, row_size,
                                  num_vals_limit, (hipStream_t)s);
}

}  // extern "C"
