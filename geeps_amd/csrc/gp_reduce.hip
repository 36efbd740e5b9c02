// gp_reduce.hip — the C-ABI (include/gp_reduce.h) of the GeePS
// gradient-update reduction path on gfx950 (MI355X / CDNA4), except the
// unplanned row calls: the N-way bucket sums (the server's apply_updates,
// src/server/tablet-server.cpp:119-134), the row plans (a fixed DoubleIndex
// compiled once: libgeeps' Update / Read), the assign and segmented row calls,
// the HBM probe, launch-plan queries, and the thread's error message.
//
// The kernels themselves (bucket_sum_*_kernel, row_*_kernel) and their launch
// logic are in gp_kernels.hpp, shared with gp_unplanned.hip (the reference
// binding's unplanned calls and their device planning).  The library's other
// translation units: gp_sort.hip (hipCUB radix sort), gp_runtime.hip (runtime
// helpers and IPC, no kernels), gp_host.cpp (the host row ops).
//
// All of it is HBM-bandwidth bound (elementwise fp32 add, row moves; no MFMA:
// there is no contraction).  Wave64 throughout: 256-thread workgroups = 4
// waves, one per SIMD.

#include "gp_kernels.hpp"

namespace {

thread_local std::string g_last_error;  // gp_last_error(), set through gp_internal::set_error

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

}  // namespace

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
namespace {

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

int create_plan(gp_row_plan *plan, const gp_double_index *host_index, size_t num_rows,
                gp_double_index offset, size_t row_size, size_t num_vals_limit, bool gather);

}  // namespace

// ===========================================================================
// C-ABI
// ===========================================================================
extern "C" {

int gp_abi_version(void) { return GP_ABI_VERSION; }

const char *gp_last_error(void) { return g_last_error.c_str(); }

int gp_scatter_rows(float *y, const float *x, const gp_double_index *index,
                    size_t num_rows, gp_double_index offset, size_t row_size,
                    size_t num_vals_limit, gp_stream s) {
  return launch_row_op<kAssignFrom>(y, x, index, num_rows, offset, row_size,
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

// The thread's gp_last_error message, set by every translation unit of the
// library (gp_kernels.hpp's set_error, in this file and gp_unplanned.hip;
// gp_host.cpp: host-memory row ops; gp_runtime.hip: memory, streams, events,
// IPC).
namespace gp_internal {
int set_error(int code, const char *msg) {
  g_last_error = msg;
  return code;
}
}  // namespace gp_internal
