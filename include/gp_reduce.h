/*
 * gp_reduce.h — C-ABI of the MI355X (gfx950) gradient-update reduction path.
 *
 * This is the thin boundary between host code (the C++ libgeeps in
 * geeps_amd/csrc/geeps, the Python test/bench harness through ctypes) and the
 * hand-written HIP kernels in geeps_amd/csrc/gp_reduce.hip.  Plain pointers and
 * sizes only; no HIP, torch or C++ types cross it.
 *
 * Every entry point replaces one reference function (GeePS, cuihenggang/geeps);
 * the reference file:line is cited next to it.  Argument meaning follows the
 * reference exactly (same index semantics, same `num_vals_limit` guard, same
 * summation order).  Differences that are deliberate:
 *   - sizes are 64-bit throughout (the reference's `int n` / `int i` grid-stride
 *     loops overflow past 2^31 elements: src/common/gpu-util/mkl_alternate.hpp:62,
 *     src/common/gpu-util/device_alternate.hpp:31-54);
 *   - calls are asynchronous on the given stream (the reference synchronises
 *     after every launch: src/common/row-op-util.cu:141); the caller syncs.
 *     The one exception: a large unplanned row call (gp_scatter_add_rows and
 *     kin, >= gp_set_unplanned_min_bytes) waits for its stream once on the
 *     first call with an index (the device scan's summary; also on the second
 *     for a scatter of rows over 128 floats, which sorts then); later calls
 *     with the same index are asynchronous too (ABI 11, 12);
 *   - errors are returned as a status code (0 = GP_OK) with a thread-local
 *     message from gp_last_error(), instead of a glog FATAL abort
 *     (src/common/gpu-util/device_alternate.hpp:16-28).  The C++ layer above
 *     turns a non-zero status into an abort with that message.
 *
 * All functions are re-entrant.  Global state: the thread-local error string,
 * per-device / per-kernel launch facts cached on first use (CU count,
 * resident blocks per CU), which never change once read, and the unplanned
 * calls' plan cache (mutex-protected; see gp_unplanned_cache_clear).
 */
#ifndef GP_REDUCE_H_
#define GP_REDUCE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Status codes. */
#define GP_OK 0
#define GP_ERR_INVALID 1   /* bad argument (null pointer, zero row size ...) */
#define GP_ERR_HIP 2       /* a HIP runtime call failed */
#define GP_ERR_UNSUPPORTED 3

/* Library ABI version; bumped on any signature change. */
#define GP_ABI_VERSION 16

/* {id0, id1} pair, 16 bytes, identical layout to the reference's
 * `struct DoubleIndex { size_t id0; size_t id1; }`
 * (src/common/row-op-util.hpp:40-44).  id0 = row position in the app's op
 * buffer, id1 = row in the process/param cache
 * (src/client/clientlib-viter.cpp:841). */
typedef struct gp_double_index {
  uint64_t id0;
  uint64_t id1;
} gp_double_index;

/* An opaque hipStream_t.  NULL = the device's null stream. */
typedef void *gp_stream;
/* An opaque hipEvent_t. */
typedef void *gp_event;

int gp_abi_version(void);
const char *gp_last_error(void);
/* ABI 10: the size from which gp_scatter_add_rows / gp_scatter_init_rows /
 * gp_gather_rows plan themselves on the device (num_rows * row_size * 4
 * bytes; default 64 MiB; SIZE_MAX: never).  Process-wide; for tests and
 * measurement. */
int gp_set_unplanned_min_bytes(size_t min_bytes);
/* The unplanned calls' plan cache (ABI 10, 11): a large call keeps its plan
 * for later calls with the same index (same pointer, size, offsets, row size
 * and limit, and the same content, which every such call checks entry for
 * entry on the device): a copy of the index and a 4-B compact copy of each
 * entry's id1, its dense runs and its residual -- as an inverse map over
 * destination rows or in destination order when a scatter's residual is
 * unsorted, else as ranges of the index itself: 20-36 B of HBM per row, at
 * most 256 indexes and
 * gp_set_unplanned_cache_bytes() of HBM (default 4 GiB; 0 keeps nothing),
 * least recently used first out.  Clear it, read its size, or bound it. */
int gp_unplanned_cache_clear(void);
int gp_unplanned_cache_entries(size_t *entries, size_t *bytes);
int gp_set_unplanned_cache_bytes(size_t max_bytes);
/* What the unplanned calls' planning did since the process started (ABI 12;
 * process-wide counters, for tests and measurement). */
typedef struct gp_unplanned_stats {
  uint64_t scans;         /* calls that scanned their index (a first call, a re-plan) */
  uint64_t steady_calls;  /* calls that ran a kept plan behind the device check */
  uint64_t stale_drops;   /* kept plans dropped: a check found the index changed, or
                             the inverse map built for it was unsound (a repeated
                             destination, a source row past 2^32) */
  uint64_t inverse_plans; /* inverse maps built (first calls) */
  uint64_t sorted_plans;  /* destination-sorted residuals built (second calls) */
  uint64_t ranges_plans;  /* ranges plans kept (first calls) */
} gp_unplanned_stats;
int gp_unplanned_stats_get(gp_unplanned_stats *out);

/* ---------------------------------------------------------------------------
 * Row operations (client side).  Element (row r, value v) lives at
 * base[r * row_size + v].  `row_size` is a runtime argument (the public API
 * fixes it at 128 floats, ROW_DATA_SIZE in geeps-user-defined-types.hpp:54).
 * ------------------------------------------------------------------------- */

/* Row-indexed scatter-add (the client delta accumulate):
 *   for r in [0, num_rows), v in [0, row_size):
 *     from = index[r].id0 + offset.id0;  to = index[r].id1 + offset.id1;
 *     if (from*row_size + v < num_vals_limit)
 *       y[to*row_size + v] += x[from*row_size + v];
 * Replaces add_rows_from_double_index_gpu (src/common/row-op-util.hpp:151-155,
 * src/common/row-op-util.cu:109-142); CPU twin add_rows_from_double_index_cpu
 * (src/common/row-op-util.hpp:121-139).
 * Precondition (as for the reference kernel, whose threads race on a repeated
 * destination): destination rows index[r].id1 are distinct within one call.
 * `index` is a DEVICE pointer.  num_rows == 0 is a no-op.
 * Calls of at least gp_set_unplanned_min_bytes() of rows (default 64 MiB)
 * plan themselves on the device (ABI 10-12): one pass over the index finds its
 * dense runs (moved like a row plan's, by the phase-separated sum kernels) and
 * whether the other rows' destinations ascend; if they do not, rows of up to
 * 128 floats go through an inverse map over destination rows, built by the
 * same call (wider rows: op order, and the next call with the same index
 * builds a destination-sorted copy of them).  A first call waits for the
 * stream once, for the index summary, as the reference's call waits at its end
 * (row-op-util.cu:141).  Later calls with the same index (ABI 11) do not: the
 * device compares the index with the kept copy and runs the kept plan if it is
 * unchanged, the op-order form if not, with no host round trip.  Smaller
 * calls are fully asynchronous.  Same results every way
 * (gp_unplanned_cache_clear, gp_unplanned_stats_get). */
int gp_scatter_add_rows(float *y, const float *x, const gp_double_index *index,
                        size_t num_rows, gp_double_index offset,
                        size_t row_size, size_t num_vals_limit, gp_stream s);

/* Fused zerofy + scatter-add for a destination the call's rows cover:
 *     y[to*row_size + v] = 0.0f + x[from*row_size + v]   (from*row_size+v < limit)
 *     y[to*row_size + v] = 0.0f                          (otherwise)
 * for every listed row — bit-identical, per listed destination row, to
 * DataStorage::zerofy_data_gpu (common-util.hpp:445-456) followed by
 * gp_scatter_add_rows (0.0f + x maps -0.0 to +0.0 exactly as the add does).
 * Destinations NOT listed are left untouched (not zeroed): the caller uses it
 * only when the clock's update ops cover every oplog row exactly once
 * (client_viter.cpp, FinishVirtualIteration).  Same index semantics, precondition
 * and large-call planning as gp_scatter_add_rows. */
int gp_scatter_init_rows(float *y, const float *x, const gp_double_index *index,
                         size_t num_rows, gp_double_index offset,
                         size_t row_size, size_t num_vals_limit, gp_stream s);

/* Row-indexed gather (the Read path, refresh leg):
 *     from = index[r].id1 + offset.id1;  to = index[r].id0 + offset.id0;
 *     if (to*row_size + v < num_vals_limit)
 *       y[to*row_size + v] = x[from*row_size + v];
 * Replaces assign_rows_to_double_index_gpu (src/common/row-op-util.hpp:141-145,
 * src/common/row-op-util.cu:39-72); CPU twin :81-99.  Large calls plan
 * themselves as gp_scatter_add_rows does (dense runs copied by the sweep). */
int gp_gather_rows(float *y, const float *x, const gp_double_index *index,
                   size_t num_rows, gp_double_index offset, size_t row_size,
                   size_t num_vals_limit, gp_stream s);

/* Row-indexed scatter-assign:
 *     from = index[r].id0 + offset.id0;  to = index[r].id1 + offset.id1;
 *     if (from*row_size + v < num_vals_limit)
 *       y[to*row_size + v] = x[from*row_size + v];
 * Replaces assign_rows_from_double_index_gpu (src/common/row-op-util.hpp:146-150,
 * src/common/row-op-util.cu:74-107; no callers in the reference). */
int gp_scatter_rows(float *y, const float *x, const gp_double_index *index,
                    size_t num_rows, gp_double_index offset, size_t row_size,
                    size_t num_vals_limit, gp_stream s);

/* ---------------------------------------------------------------------------
 * Row plans: a scatter DoubleIndex compiled once, for ops whose index is fixed
 * (libgeeps builds one per op and channel at FinishVirtualIteration, where the
 * reference builds the op's device DoubleIndex: vi_create_double_index,
 * src/client/clientlib-viter.cpp:817-883).  The plan visits the rows in
 * destination (id1) order -- bit-neutral, since each row's adds keep their
 * order: a destination listed more than once (the reference's channel check,
 * range == count at clientlib-viter.cpp:869-873, admits e.g. cache rows
 * {0, 0, 2}) gets its later occurrences from "repeat layers" that run after
 * the first occurrences, one layer per occurrence, so its adds land in op
 * order as in the CPU twin add_rows_from_double_index_cpu
 * (src/common/row-op-util.hpp:121-139).  (The reference's GPU kernel races on
 * such a row; the unplanned gp_scatter_add_rows keeps its precondition.)
 * Runs in which id0 and id1 both step by one (whole rows, at least 4 MiB) are
 * moved as dense ranges by the phase-separated sum kernels (the init by their
 * zero-input form); the other rows
 * keep a device index, sorted by id1, for the row kernels, so the scatter's
 * read-modify-write side walks y front to back.  Results are bit-identical to
 * gp_scatter_add_rows / gp_scatter_init_rows over the same index, offset and
 * num_vals_limit.
 * ------------------------------------------------------------------------- */
typedef struct gp_row_plan_s *gp_row_plan;

/* Build a plan from a HOST copy of `num_rows` DoubleIndex entries; `offset`
 * and `num_vals_limit` are baked in (same meaning as gp_scatter_add_rows).
 * The plan's device index lives on the current device, and the plan runs only
 * there. */
int gp_row_plan_create(gp_row_plan *plan, const gp_double_index *host_index, size_t num_rows,
                       gp_double_index offset, size_t row_size, size_t num_vals_limit);
int gp_row_plan_destroy(gp_row_plan plan);
/* The plan's rows, its dense runs and the rows in them (the rest go to the
 * row kernels). */
int gp_row_plan_info(gp_row_plan plan, size_t *num_rows, size_t *dense_runs, size_t *dense_rows);
/* ABI 10: the plan's repeat layers (0 when every destination is distinct) and
 * the rows in them (each destination's second, third ... occurrence). */
int gp_row_plan_repeats(gp_row_plan plan, size_t *layers, size_t *repeat_rows);
/* Launch plan of one planned add (init = 0) or fused init (init = 1) over
 * 16-B-aligned buffers (a gather plan: its gather, `init` ignored, flat
 * cache); launches nothing.  *sweep_launches = launches of the
 * stream-by-stream sum kernel over the dense runs (1 bucket; the init's
 * zero-input form), *phased_launches = tile-major phase-separated launches,
 * *other_launches = everything else (mixed / scalar sum forms, one row
 * kernel launch for the residual rows and one per repeat layer).  For
 * measurement tools (bench.py). */
int gp_row_plan_launches(gp_row_plan plan, int init, int *sweep_launches, int *phased_launches,
                         int *other_launches);
/* gp_scatter_add_rows(y, x, index, ...) through the plan (a3:
 * add_rows_from_double_index_gpu, src/common/row-op-util.cu:109-142). */
int gp_scatter_add_rows_planned(float *y, const float *x, gp_row_plan plan, gp_stream s);
/* gp_scatter_init_rows(y, x, index, ...) through the plan (a7 + a3: the fused
 * zerofy_data_gpu + add, common-util.hpp:445-456). */
int gp_scatter_init_rows_planned(float *y, const float *x, gp_row_plan plan, gp_stream s);

/* ---------------------------------------------------------------------------
 * Segmented param cache.  The cache rows of one table are split into up to
 * GP_MAX_SEGMENTS contiguous row ranges, each living in its own buffer: range
 * i is rows [first_row[i], first_row[i+1]) (the last one open-ended) and cache
 * row c of range i is at base[i][(c - first_row[i]) * row_size].  libgeeps
 * uses it so a refreshed shard is read in place from the server's published
 * master version (its own buffer, or an IPC mapping of a same-node server's)
 * instead of being copied into one contiguous cache first; the reference has
 * one contiguous cache (ParamCache::data_cache, clientlib.hpp:338-341).
 * first_row[0] must be 0 and first_row strictly ascending.
 * ------------------------------------------------------------------------- */
#define GP_MAX_SEGMENTS 64

typedef struct gp_row_segments {
  uint32_t count; /* 1 .. GP_MAX_SEGMENTS */
  uint32_t reserved;
  uint64_t first_row[GP_MAX_SEGMENTS];
  float *base[GP_MAX_SEGMENTS];
} gp_row_segments;

/* gp_gather_rows with x = the segmented cache: `from` (id1 + offset.id1) is a
 * cache row resolved through `x_segments`. */
int gp_gather_rows_segmented(float *y, const gp_row_segments *x_segments,
                             const gp_double_index *index, size_t num_rows,
                             gp_double_index offset, size_t row_size,
                             size_t num_vals_limit, gp_stream s);

/* gp_scatter_add_rows with y = the segmented cache: `to` (id1 + offset.id1)
 * is a cache row resolved through `y_segments` (read-my-writes: the update
 * also lands in the param cache, clientlib-data.cpp:387-392). */
int gp_scatter_add_rows_segmented(const gp_row_segments *y_segments, const float *x,
                                  const gp_double_index *index, size_t num_rows,
                                  gp_double_index offset, size_t row_size,
                                  size_t num_vals_limit, gp_stream s);

/* A GATHER plan: the same compilation for gp_gather_rows' index (y[id0] =
 * x[id1], assign_rows_to_double_index_gpu, src/common/row-op-util.cu:39-72:
 * num_vals_limit guards the destination y).  libgeeps builds one per Read op
 * and channel.  Rows are visited in destination (id0) order (a repeated
 * destination through repeat layers in op order: the last one listed wins, as
 * in the CPU twin's loop); dense runs are plain copies
 * through the phase-separated kernels, the rest goes to the gather row
 * kernels.  A gather plan works only with the gp_gather_rows_*planned calls,
 * a scatter plan only with the scatter ones (GP_ERR_INVALID otherwise). */
int gp_gather_plan_create(gp_row_plan *plan, const gp_double_index *host_index, size_t num_rows,
                          gp_double_index offset, size_t row_size, size_t num_vals_limit);
/* gp_gather_rows(y, x, index, ...) through a gather plan. */
int gp_gather_rows_planned(float *y, const float *x, gp_row_plan plan, gp_stream s);
/* gp_gather_rows_segmented(y, x_segments, index, ...) through a gather plan:
 * a dense run that crosses a segment boundary is copied piece by piece. */
int gp_gather_rows_segmented_planned(float *y, const gp_row_segments *x_segments, gp_row_plan plan,
                                     gp_stream s);

/* ---------------------------------------------------------------------------
 * Dense reductions (server side).
 * ------------------------------------------------------------------------- */

/* N-way bucket sum applied to the master shard, in bucket order:
 *     for i in [0, num_vals):
 *       master[i] = (((master[i] + b[0][i]) + b[1][i]) + ...) + b[N-1][i]
 * which is bit-identical to the reference server applying N client messages
 * in arrival order 0..N-1, each one `cpu_add(n, master, update, master)`
 * (TabletStorage::apply_updates, src/server/tablet-server.cpp:119-134 ->
 * cpu_add<float>, src/common/gpu-util/math_functions.cpp:132-136 -> vsAdd,
 * src/common/gpu-util/mkl_alternate.hpp:59-74).
 * `buckets` is a HOST array of `num_buckets` DEVICE pointers.
 * num_buckets == 0 or num_vals == 0 is a no-op.  Every byte moves once per
 * pass of up to 8 buckets: (N + 1) * num_vals * 4 B read, num_vals * 4 B
 * written, in one launch per phase-separated chunk (gp_bucket_sum_plan).
 * More than 8 buckets: consecutive passes continue the bucket order. */
int gp_bucket_sum_apply(float *master, const float *const *buckets,
                        int num_buckets, size_t num_vals, gp_stream s);

/* Out-of-place form of gp_bucket_sum_apply:
 *     out[i] = (((in[i] + b[0][i]) + b[1][i]) + ...) + b[N-1][i]
 * with `in` left unchanged (same bits as applying the N buckets to a copy of
 * `in`).  libgeeps' tablet server uses it to build the next version of a
 * shard while clients still read the last published one in place (the
 * refresh the reference sends as a copy, server-encoder-decoder.cpp:228-250).
 * `out` and `in` must not overlap unless equal (then it is
 * gp_bucket_sum_apply).  Same traffic as the in-place form.
 * num_buckets == 0 copies `in` to `out`. */
int gp_bucket_sum_into(float *out, const float *in, const float *const *buckets,
                       int num_buckets, size_t num_vals, gp_stream s);

/* Launch plan of ONE pass of gp_bucket_sum_apply / _into with num_buckets
 * (1..8) over num_vals floats in 16-B-aligned buffers; launches nothing.
 * *phased_launches = launches of the phase-separated kernels, sweep and
 * tile-major together (0 when the shard is too small for them and the mixed
 * form sums it in one launch);
 * *reg_tiles = tiles per block held in registers beside the 160 KiB in LDS
 * by the first phased form (sweep, 96-MiB chunks: 7 tiles of 32 KiB at 2-8
 * buckets, 14 of 16 KiB at 1; 64-MiB chunks: 6 of 16 KiB; tile-major: 20 at
 * 1-2 buckets, 12 at 3-4, 4 at 5-8, of 16 KiB; -1: not phased).  For
 * measurement tools: bench.py prices the dominant kernel per launch with it,
 * as rocprofv3 reports it.
 * Returns GP_ERR_INVALID for num_buckets outside 1..8. */
int gp_bucket_sum_plan(size_t num_vals, int num_buckets, int *phased_launches,
                       int *reg_tiles);

/* The same plan, plus *sweep_launches = how many of the phased launches are
 * the stream-by-stream sweep kernel, big and small chunks together
 * (gp_bucket_sum_launch_plan splits them); *reg_tiles is then the first sweep
 * form's: 7 or 14 (96-MiB chunks) or 6 (64-MiB chunks). */
int gp_bucket_sum_sweep_plan(size_t num_vals, int num_buckets, int *phased_launches,
                             int *reg_tiles, int *sweep_launches);

/* Every launch of one pass of num_buckets (1..8) over num_vals floats in
 * 16-B-aligned buffers, by kernel form, in launch order; launches nothing:
 *   sweep_launches       the stream-by-stream kernel's big chunks (96 MiB on
 *                        256 CUs: 384 KiB per block, 160 KiB of it in LDS;
 *                        sweep_reg_tiles tiles of sweep_tile_kib KiB in
 *                        registers, bursts of sweep_burst_tiles tiles: 7 x 32
 *                        KiB, bursts of 1, at 2-8 buckets; 14 x 16 KiB, bursts
 *                        of 8, at 1),
 *   small_sweep_launches then its 64-MiB chunks (6 register tiles, bursts of
 *                        small_sweep_burst_tiles = 4),
 *   phased_launches      then the tile-major phase-separated form
 *                        (phased_reg_tiles: 20 at 1-2 buckets, 12 at 3-4, 4 at 5-8),
 *   other_launches       then the mixed dwordx4 and scalar forms (0-2).
 * A reg_tiles / burst_tiles field is -1 when its form has no launch.  For
 * measurement tools: bench.py names and prices each kernel instantiation per
 * launch (bucket_sum_sweep_kernel<NB, reg_tiles, burst_tiles, zin, strides>), as
 * rocprofv3 reports it. */
typedef struct gp_sum_plan {
  int sweep_launches, sweep_reg_tiles;
  int small_sweep_launches;
  int phased_launches, phased_reg_tiles;
  int other_launches;
  int sweep_burst_tiles, small_sweep_burst_tiles; /* ABI 9 */
  int sweep_tile_kib;                              /* ABI 9: 16 or 32 */
} gp_sum_plan;
int gp_bucket_sum_launch_plan(size_t num_vals, int num_buckets, gp_sum_plan *plan);

/* y[i] = a[i] + b[i] — device form of cpu_add / vsAdd
 * (src/common/gpu-util/math_functions.hpp:60-61, mkl_alternate.hpp:59-74).
 * Also covers add_row_batch_gpu's `y += x` (cublasSaxpy with alpha 1,
 * src/common/row-op-util.hpp:72-79) as gp_add(n, y, x, y). In-place allowed. */
int gp_add(size_t n, const float *a, const float *b, float *y, gp_stream s);

/* HBM probe for measurement tools: stream `num_vals` floats of a 16-B
 * aligned device buffer once, read-only (GP_PROBE_READ: 16-B non-temporal
 * loads; the buffer is not written) or write-only (GP_PROBE_WRITE: zeros,
 * through the runtime's fill kernel).
 * bench.py times both to model every kernel's bytes on the same box.  No
 * reference counterpart. */
#define GP_PROBE_READ 0
#define GP_PROBE_WRITE 1
int gp_hbm_probe(int kind, float *buffer, size_t num_vals, gp_stream s);

/* Zero `num_vals` floats — DataStorage::zerofy_data_gpu
 * (src/common/common-util.hpp:445-456). */
int gp_zero(float *y, size_t num_vals, gp_stream s);

/* ---------------------------------------------------------------------------
 * Host-memory row ops: the reference's CPU twins, for rows a GeePS param cache
 * keeps in host memory.  When `gpu_memory_capacity` cannot hold every row, the
 * reference places whole key batches in a CPU param cache
 * (vi_decide_param_cache, src/client/clientlib-viter.cpp:492-611) and runs
 * these loops there (update_batch_cpu / read_batch_cpu / recv_row_batch_cpu,
 * src/client/clientlib-data.cpp:153-189, 280-302, 398-434); libgeeps' host
 * tier does the same with these (ABI 13).  Synchronous, on the calling
 * thread; same index, offset, `num_vals_limit` and order semantics as the
 * reference loops (entries in index order, so a repeated destination gets
 * its adds in op order).  Pure host code: no device, stream or HIP runtime.
 * ------------------------------------------------------------------------- */
/* y[(id1+off1)*W + v] += x[(id0+off0)*W + v] where (id0+off0)*W + v < limit
 * -- add_rows_from_double_index_cpu (src/common/row-op-util.hpp:121-139). */
int gp_host_scatter_add_rows(float *y, const float *x, const gp_double_index *index, size_t num_rows,
                             gp_double_index offset, size_t row_size, size_t num_vals_limit);
/* The fused zerofy + scatter-add (ABI 15): the same bits as zerofy_data_cpu
 * of the listed destination rows, then add_rows_from_double_index_cpu.  A
 * destination's first entry writes 0.0f + x[(id0+off0)*W + v] (0.0f where
 * that x index is at or past the limit), later ones add, in entry order.
 * libgeeps' host tier uses it when a clock's update ops write every host
 * oplog row once: the oplog is then never zeroed. */
int gp_host_scatter_init_rows(float *y, const float *x, const gp_double_index *index, size_t num_rows,
                              gp_double_index offset, size_t row_size, size_t num_vals_limit);
/* y[(id0+off0)*W + v] = x[(id1+off1)*W + v] where (id0+off0)*W + v < limit
 * -- assign_rows_to_double_index_cpu (src/common/row-op-util.hpp:81-99). */
int gp_host_gather_rows(float *y, const float *x, const gp_double_index *index, size_t num_rows,
                        gp_double_index offset, size_t row_size, size_t num_vals_limit);
/* y[i] += x[i], i < n -- add_row_batch (src/common/row-op-util.hpp:64-70,
 * cpu_axpy with alpha 1: the same bits as one fp32 add per element). */
int gp_host_add(size_t n, float *y, const float *x);
/* y[i] = 0, i < n -- zerofy_data_cpu (src/common/common-util.hpp:437-443),
 * threaded like the row ops for large buffers (a host oplog of a large table
 * is zeroed every clock). */
int gp_host_zero(size_t n, float *y);

/* ---------------------------------------------------------------------------
 * Runtime helpers, so host C++ never names a HIP type.
 * ------------------------------------------------------------------------- */
int gp_device_count(int *count);
int gp_set_device(int device);
int gp_get_device(int *device);
/* Device memory; buffers of 64 MiB and up are requested physically
 * contiguous first (steadier HBM rates for the streaming sums), plain
 * otherwise or when no contiguous range is left. */
int gp_malloc_device(void **ptr, size_t bytes);
/* A device buffer that may be exported over IPC (gp_ipc_get_handle): an
 * allocation of its own, at least `bytes` + 256 rounded up to a multiple of
 * 2 MiB; its last 256 bytes hold the export's tag (ABI 11).  Free with
 * gp_free_device. */
int gp_malloc_device_shared(void **ptr, size_t bytes);
int gp_free_device(void *ptr);
int gp_malloc_host(void **ptr, size_t bytes); /* pinned (mallocHost) */
int gp_free_host(void *ptr);
/* Page-lock an existing host range, and undo it (ABI 14): libgeeps' host-tier
 * oplogs are shared memory mapped into a same-node peer process as well
 * (DESIGN.md §4.1); each process registers its own mapping so that copies
 * between it and HBM run at the pinned PCIe rate.  Unregister before unmapping. */
int gp_host_register(void *ptr, size_t bytes);
int gp_host_unregister(void *ptr);
/* Direction inferred from the pointers (cudaMemcpyDefault in the reference). */
int gp_memcpy_async(void *dst, const void *src, size_t bytes, gp_stream s);
int gp_memset_async(void *dst, int value, size_t bytes, gp_stream s);
int gp_stream_create(gp_stream *s);      /* non-blocking stream */
int gp_stream_destroy(gp_stream s);
int gp_stream_synchronize(gp_stream s);
int gp_device_synchronize(void);
int gp_event_create(gp_event *e);
int gp_event_destroy(gp_event e);
int gp_event_record(gp_event e, gp_stream s);
int gp_event_synchronize(gp_event e);
int gp_event_elapsed_ms(float *ms, gp_event start, gp_event stop);
/* Work queued on `s` after this call waits for `e`'s last record. */
int gp_stream_wait_event(gp_stream s, gp_event e);
/* The device's PCI bus id ("0000:05:00.0"), NUL-terminated in buf[len]: a
 * name of the physical GPU that is the same in every process, whatever
 * device numbering (HIP_VISIBLE_DEVICES) each one sees. */
int gp_device_pci_bus_id(int device, char *buf, int len);

/* Inter-process device memory (same node; xGMI between MI355X devices):
 * export the BASE of a gp_malloc_device_shared buffer (anything else is
 * refused with GP_ERR_INVALID) as an opaque handle, map a peer's handle into
 * this process (peer access enabled lazily), unmap.  ABI 11: the export
 * writes a tag into the buffer's spare end and the handle carries it; a
 * mapping that does not hold it (the runtime mapped other memory) fails with
 * GP_ERR_HIP instead of handing out wrong rows. */
#define GP_IPC_HANDLE_BYTES 96
int gp_ipc_get_handle(void *handle_out, void *device_base);
/* ABI 16: a mapping that fails the tag check is left mapped and never used
 * (unmapped, its address could go to a buffer this process exports later,
 * which the runtime may then resolve to stale memory: DESIGN.md §4), and the
 * error names what the handle names, what the mapping held and the raw
 * runtime handle; after 16 such mis-mappings in one process every later open
 * is refused (GP_ERR_HIP). */
int gp_ipc_open_handle(void **device_ptr, const void *handle);
int gp_ipc_close_handle(void *device_ptr);
/* ABI 16: one line on a handle (NUL-terminated in buf[len]): the exporter's
 * pid, buffer base and size as libgeeps recorded them, the process and
 * address the runtime's handle names, and whether the two agree. */
int gp_ipc_describe_handle(const void *handle, char *buf, int len);
/* ABI 16: this process's mis-mapped opens so far (each left mapped, unused). */
int gp_ipc_mismaps(int *count);

#ifdef __cplusplus
}  /* extern "C" */
#endif

#endif  /* GP_REDUCE_H_ */
