/*
 * c_abi_check.c — a plain C99 consumer of the C-ABI (include/gp_reduce.h).
 *
 * TEST PROGRAM.  It proves the boundary is what INTEGRATION.md says it is: a C
 * header with plain pointers and sizes that a C (or cgo / FFI) caller can use
 * with no HIP, C++ or torch type in sight.  Built by __graft_entry__.build()
 * with `gcc -std=c99 -pedantic -Wall -Wextra -Werror`, linked against
 * libgp_reduce.so (the product) and oracle/build/liboracle.so (the checker,
 * test infrastructure: only tests/ link it).  tests/test_abi.py checks that it
 * builds (CPU); tests/test_gpu_parity.py runs it on the GPU.
 *
 * Cases, each checked bit for bit against the oracle's restatement of the
 * reference arithmetic:
 *   1. gp_bucket_sum_apply: 8 buckets into a master of 5 Mi + 3 floats
 *      (TabletStorage::apply_updates x 8 in arrival order,
 *      src/server/tablet-server.cpp:119-134);
 *   2. gp_scatter_add_rows: a random permutation DoubleIndex with an offset
 *      and a num_vals_limit that cuts a row (add_rows_from_double_index_gpu,
 *      src/common/row-op-util.cu:109-142);
 *   3. the same index through a row plan (gp_scatter_add_rows_planned) and its
 *      fused init (zerofy_data_gpu + add);
 *   4. gp_gather_rows and a gather plan (assign_rows_to_double_index_gpu,
 *      src/common/row-op-util.cu:39-72);
 *   5. the error convention: a null pointer returns GP_ERR_INVALID with a
 *      message from gp_last_error(), an unknown bucket count likewise.
 * Prints "c_abi_check ok" and exits 0; any mismatch exits 1.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gp_reduce.h"

/* oracle/oracle.c (no header: test infrastructure) */
int oracle_apply_updates(float *master, const float *const *updates, int n_clients,
                         int64_t num_vals);
void oracle_add_rows_from_double_index(float *y, const float *x, const uint64_t *index,
                                       size_t num_rows, uint64_t off0, uint64_t off1,
                                       size_t row_size, size_t num_vals_limit);
void oracle_assign_rows_to_double_index(float *y, const float *x, const uint64_t *index,
                                        size_t num_rows, uint64_t off0, uint64_t off1,
                                        size_t row_size, size_t num_vals_limit);

static int failures = 0;

#define CALL(expr)                                                                   \
  do {                                                                               \
    int rc_ = (expr);                                                                \
    if (rc_ != GP_OK) {                                                              \
      fprintf(stderr, "%s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #expr, rc_,        \
              gp_last_error());                                                      \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

static uint64_t rng_state = 0x9e3779b97f4a7c15ull;

static uint64_t next_u64(void) {
  uint64_t z = (rng_state += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

/* uniform in [-0.5, 0.5), with a few signed zeros (0.0f + -0.0f = +0.0f must hold) */
static void fill(float *p, size_t n) {
  size_t i;
  for (i = 0; i < n; ++i) p[i] = (float)((next_u64() >> 40) * (1.0 / 16777216.0)) - 0.5f;
  if (n > 2) {
    p[0] = -0.0f;
    p[n / 2] = -0.0f;
  }
}

static void *dev_alloc(size_t bytes) {
  void *p = NULL;
  CALL(gp_malloc_device(&p, bytes));
  return p;
}

static void to_dev(void *d, const void *h, size_t bytes) {
  CALL(gp_memcpy_async(d, h, bytes, NULL));
  CALL(gp_stream_synchronize(NULL));
}

static void to_host(void *h, const void *d, size_t bytes) {
  CALL(gp_memcpy_async(h, d, bytes, NULL));
  CALL(gp_stream_synchronize(NULL));
}

static void expect_same(const char *what, const float *got, const float *want, size_t n) {
  size_t i, bad = 0, first = 0;
  for (i = 0; i < n; ++i)
    if (memcmp(&got[i], &want[i], sizeof(float)) != 0) {
      if (!bad) first = i;
      ++bad;
    }
  if (bad) {
    fprintf(stderr, "%s: %zu of %zu values differ (first at %zu: %a vs %a)\n", what, bad, n,
            first, (double)got[first], (double)want[first]);
    ++failures;
  } else {
    printf("%s: %zu values bit-exact\n", what, n);
  }
}

static void bucket_sum_case(void) {
  const size_t n = (size_t)5 * 1024 * 1024 + 3;
  const int nb = 8;
  float *h_master = malloc(n * sizeof(float)), *h_want = malloc(n * sizeof(float));
  float *h_b[8], *d_b[8], *d_master;
  const float *want_b[8];
  const float *dev_b[8];
  int k;
  fill(h_master, n);
  memcpy(h_want, h_master, n * sizeof(float));
  d_master = dev_alloc(n * sizeof(float));
  to_dev(d_master, h_master, n * sizeof(float));
  for (k = 0; k < nb; ++k) {
    h_b[k] = malloc(n * sizeof(float));
    fill(h_b[k], n);
    d_b[k] = dev_alloc(n * sizeof(float));
    to_dev(d_b[k], h_b[k], n * sizeof(float));
    want_b[k] = h_b[k];
    dev_b[k] = d_b[k];
  }
  CALL(gp_bucket_sum_apply(d_master, dev_b, nb, n, NULL));
  to_host(h_master, d_master, n * sizeof(float));
  oracle_apply_updates(h_want, want_b, nb, (int64_t)n);
  expect_same("gp_bucket_sum_apply 8 buckets", h_master, h_want, n);
  for (k = 0; k < nb; ++k) {
    CALL(gp_free_device(d_b[k]));
    free(h_b[k]);
  }
  CALL(gp_free_device(d_master));
  free(h_master);
  free(h_want);
}

static void row_cases(void) {
  const size_t W = 128, rows = 40000, cache_rows = rows + 7;
  const uint64_t off0 = 3, off1 = 5;
  /* the limit cuts source row (rows - 2) + off0 halfway: its tail is skipped */
  const size_t limit = ((rows - 2) + off0) * W + W / 2;
  const size_t x_vals = (rows + off0) * W, y_vals = (cache_rows + off1) * W;
  uint64_t *idx = malloc(rows * 2 * sizeof(uint64_t));
  float *hx = malloc(x_vals * sizeof(float)), *hy = malloc(y_vals * sizeof(float));
  float *want = malloc(y_vals * sizeof(float)), *got = malloc(y_vals * sizeof(float));
  float *dx, *dy;
  gp_double_index *didx;
  gp_double_index off;
  gp_row_plan plan = NULL;
  size_t r, i;
  off.id0 = off0;
  off.id1 = off1;

  /* id0 = r, id1 = a random permutation of the cache rows' first `rows` */
  for (r = 0; r < rows; ++r) {
    idx[2 * r] = r;
    idx[2 * r + 1] = r;
  }
  for (r = rows - 1; r > 0; --r) {
    const size_t j = (size_t)(next_u64() % (r + 1));
    const uint64_t t = idx[2 * r + 1];
    idx[2 * r + 1] = idx[2 * j + 1];
    idx[2 * j + 1] = t;
  }
  fill(hx, x_vals);
  fill(hy, y_vals);
  dx = dev_alloc(x_vals * sizeof(float));
  dy = dev_alloc(y_vals * sizeof(float));
  didx = dev_alloc(rows * sizeof(gp_double_index));
  to_dev(dx, hx, x_vals * sizeof(float));
  to_dev(didx, idx, rows * sizeof(gp_double_index));

  /* 2. scatter-add, device index in op order */
  to_dev(dy, hy, y_vals * sizeof(float));
  CALL(gp_scatter_add_rows(dy, dx, didx, rows, off, W, limit, NULL));
  to_host(got, dy, y_vals * sizeof(float));
  memcpy(want, hy, y_vals * sizeof(float));
  oracle_add_rows_from_double_index(want, hx, idx, rows, off0, off1, W, limit);
  expect_same("gp_scatter_add_rows", got, want, y_vals);

  /* 2b. the host-memory twin (ABI 13, the host tier): the same rows in host
   * memory through gp_host_scatter_add_rows, against the same oracle sum */
  memcpy(got, hy, y_vals * sizeof(float));
  CALL(gp_host_scatter_add_rows(got, hx, (const gp_double_index *)idx, rows, off, W, limit));
  expect_same("gp_host_scatter_add_rows", got, want, y_vals);

  /* 3. the same through a row plan: add, then fused init */
  CALL(gp_row_plan_create(&plan, (const gp_double_index *)idx, rows, off, W, limit));
  to_dev(dy, hy, y_vals * sizeof(float));
  CALL(gp_scatter_add_rows_planned(dy, dx, plan, NULL));
  to_host(got, dy, y_vals * sizeof(float));
  expect_same("gp_scatter_add_rows_planned", got, want, y_vals);

  to_dev(dy, hy, y_vals * sizeof(float));
  CALL(gp_scatter_init_rows_planned(dy, dx, plan, NULL));
  to_host(got, dy, y_vals * sizeof(float));
  memcpy(want, hy, y_vals * sizeof(float));
  for (r = 0; r < rows; ++r) /* zerofy the listed destinations, then add */
    for (i = 0; i < W; ++i) want[(idx[2 * r + 1] + off1) * W + i] = 0.0f;
  oracle_add_rows_from_double_index(want, hx, idx, rows, off0, off1, W, limit);
  expect_same("gp_scatter_init_rows_planned", got, want, y_vals);
  CALL(gp_row_plan_destroy(plan));
  /* the host-memory fused init (ABI 15) against the same zerofy + add */
  memcpy(got, hy, y_vals * sizeof(float));
  CALL(gp_host_scatter_init_rows(got, hx, (const gp_double_index *)idx, rows, off, W, limit));
  expect_same("gp_host_scatter_init_rows", got, want, y_vals);

  /* 4. gather: y[id0 + off0] = x[id1 + off1], the limit on the destination */
  {
    const size_t gy_vals = (rows + off0) * W, gx_vals = y_vals;
    const size_t glimit = ((rows - 3) + off0) * W + 17;
    float *gwant = malloc(gy_vals * sizeof(float)), *ggot = malloc(gy_vals * sizeof(float));
    float *gy = dev_alloc(gy_vals * sizeof(float)), *gx = dev_alloc(gx_vals * sizeof(float));
    fill(gwant, gy_vals);
    to_dev(gy, gwant, gy_vals * sizeof(float));
    to_dev(gx, hy, gx_vals * sizeof(float));
    CALL(gp_gather_rows(gy, gx, didx, rows, off, W, glimit, NULL));
    to_host(ggot, gy, gy_vals * sizeof(float));
    oracle_assign_rows_to_double_index(gwant, hy, idx, rows, off0, off1, W, glimit);
    expect_same("gp_gather_rows", ggot, gwant, gy_vals);

    CALL(gp_gather_plan_create(&plan, (const gp_double_index *)idx, rows, off, W, glimit));
    fill(ggot, gy_vals);
    memcpy(gwant, ggot, gy_vals * sizeof(float));
    to_dev(gy, ggot, gy_vals * sizeof(float));
    CALL(gp_gather_rows_planned(gy, gx, plan, NULL));
    to_host(ggot, gy, gy_vals * sizeof(float));
    oracle_assign_rows_to_double_index(gwant, hy, idx, rows, off0, off1, W, glimit);
    expect_same("gp_gather_rows_planned", ggot, gwant, gy_vals);
    CALL(gp_row_plan_destroy(plan));

    /* the host-memory twin (ABI 13): gp_host_gather_rows on the same rows */
    fill(ggot, gy_vals);
    memcpy(gwant, ggot, gy_vals * sizeof(float));
    CALL(gp_host_gather_rows(ggot, hy, (const gp_double_index *)idx, rows, off, W, glimit));
    oracle_assign_rows_to_double_index(gwant, hy, idx, rows, off0, off1, W, glimit);
    expect_same("gp_host_gather_rows", ggot, gwant, gy_vals);
    CALL(gp_free_device(gy));
    CALL(gp_free_device(gx));
    free(gwant);
    free(ggot);
  }

  CALL(gp_free_device(dx));
  CALL(gp_free_device(dy));
  CALL(gp_free_device(didx));
  free(idx);
  free(hx);
  free(hy);
  free(want);
  free(got);
}

static void error_cases(void) {
  gp_double_index off;
  int rc, launches = 0, tiles = 0;
  off.id0 = 0;
  off.id1 = 0;
  rc = gp_scatter_add_rows(NULL, NULL, NULL, 1, off, 128, 128, NULL);
  if (rc != GP_ERR_INVALID || gp_last_error()[0] == '\0') {
    fprintf(stderr, "null pointers: rc %d, message '%s'\n", rc, gp_last_error());
    ++failures;
  }
  rc = gp_bucket_sum_plan(1024, 9, &launches, &tiles);
  if (rc != GP_ERR_INVALID) {
    fprintf(stderr, "9 buckets per pass: rc %d\n", rc);
    ++failures;
  }
  printf("error convention: GP_ERR_INVALID + gp_last_error() ok\n");
}

int main(void) {
  int devices = 0;
  if (gp_abi_version() != GP_ABI_VERSION) {
    fprintf(stderr, "library ABI %d, header %d\n", gp_abi_version(), GP_ABI_VERSION);
    return 1;
  }
  error_cases();
  CALL(gp_device_count(&devices));
  if (devices < 1) {
    fprintf(stderr, "no GPU\n");
    return 1;
  }
  CALL(gp_set_device(0));
  bucket_sum_case();
  row_cases();
  if (failures) return 1;
  printf("c_abi_check ok\n");
  return 0;
}
