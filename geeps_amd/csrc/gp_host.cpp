// Host-memory row ops of the C-ABI (include/gp_reduce.h, ABI 13): the
// reference's CPU twins of the row ops (src/common/row-op-util.hpp:64-139),
// which libgeeps' host tier runs on the rows a param cache keeps in host
// memory past `gpu_memory_capacity` (src/client/clientlib-viter.cpp:492-611).
//
// Each loop visits the index entries in order, as the reference's does, so a
// destination listed twice gets its adds in op order.  The one change is
// shape: a whole row under the limit runs as a straight, vectorisable loop,
// and only the row that straddles `num_vals_limit` is guarded per element
// (the same elements are written with the same values either way).
#include <cstddef>
#include <cstdint>

#include "gp_reduce.h"

namespace gp_internal {
int set_error(int code, const char *msg);  // gp_reduce.hip: the thread's gp_last_error
}  // namespace gp_internal

namespace {

// Rows past num_vals_limit on the guarded side contribute nothing; a row is
// whole when its last element is under the limit.  (val_id, row_size and
// the products are 64-bit: the reference's size_t.)
template <typename F>
inline void guarded_row(size_t base, size_t row_size, size_t limit, F &&f) {
  if (base + row_size <= limit) {
    for (size_t v = 0; v < row_size; ++v) f(v);
  } else if (base < limit) {
    for (size_t v = 0; v < limit - base; ++v) f(v);
  }
}

int host_error(const char *msg) { return gp_internal::set_error(GP_ERR_INVALID, msg); }

}  // namespace

extern "C" {

int gp_host_scatter_add_rows(float *y, const float *x, const gp_double_index *index, size_t num_rows,
                             gp_double_index offset, size_t row_size, size_t num_vals_limit) {
  if (num_rows == 0) return GP_OK;
  if (!y || !x || !index || row_size == 0) return host_error("gp_host_scatter_add_rows: bad argument");
  for (size_t i = 0; i < num_rows; ++i) {
    const size_t from = index[i].id0 + offset.id0, to = index[i].id1 + offset.id1;
    const float *__restrict__ xs = x + from * row_size;
    float *__restrict__ ys = y + to * row_size;
    // the guard is on the source (x) index, row-op-util.hpp:133-135
    guarded_row(from * row_size, row_size, num_vals_limit, [&](size_t v) { ys[v] += xs[v]; });
  }
  return GP_OK;
}

int gp_host_gather_rows(float *y, const float *x, const gp_double_index *index, size_t num_rows,
                        gp_double_index offset, size_t row_size, size_t num_vals_limit) {
  if (num_rows == 0) return GP_OK;
  if (!y || !x || !index || row_size == 0) return host_error("gp_host_gather_rows: bad argument");
  for (size_t i = 0; i < num_rows; ++i) {
    const size_t from = index[i].id1 + offset.id1, to = index[i].id0 + offset.id0;
    const float *__restrict__ xs = x + from * row_size;
    float *__restrict__ ys = y + to * row_size;
    // the guard is on the destination (y, the op buffer) index, row-op-util.hpp:93-95
    guarded_row(to * row_size, row_size, num_vals_limit, [&](size_t v) { ys[v] = xs[v]; });
  }
  return GP_OK;
}

int gp_host_add(size_t n, float *y, const float *x) {
  if (n == 0) return GP_OK;
  if (!y || !x) return host_error("gp_host_add: null pointer");
  for (size_t i = 0; i < n; ++i) y[i] += x[i];
  return GP_OK;
}

}  // extern "C"
