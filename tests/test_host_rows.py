"""The C-ABI's host-memory row ops (ABI 13: gp_host_scatter_add_rows,
gp_host_gather_rows, gp_host_add) against the oracle, bit for bit, on CPU.

They are the reference's CPU twins (src/common/row-op-util.hpp:64-139), which
libgeeps' host tier runs on the key batches a param cache places in host
memory past `gpu_memory_capacity` (src/client/clientlib-viter.cpp:492-611).
Cases: identity / permuted / repeated destinations (op order), offsets,
`num_vals_limit` cutting a row mid-way and whole rows off, widths 1..1024,
empty calls, and argument rejection.
"""
import numpy as np
import pytest

from geeps_amd import rowops
from oracle import oracle


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def _index(rng, kind, n_op, n_cache):
    id0 = np.arange(n_op)
    if kind == "identity":
        id1 = np.arange(n_op)
    elif kind == "permuted":
        id1 = rng.permutation(n_cache)[:n_op]
    else:  # repeated: destinations drawn with replacement (op order matters)
        id1 = rng.integers(0, n_cache, n_op)
    return np.stack([id0, id1], 1).astype(np.int64)


@pytest.mark.parametrize("kind", ["identity", "permuted", "repeated"])
@pytest.mark.parametrize("W,limit_frac,off", [(128, None, (0, 0)), (128, 0.71, (0, 0)), (64, None, (3, 5)),
                                               (1, 0.5, (0, 0)), (1024, 0.9, (1, 2)), (7, None, (2, 0))])
def test_host_scatter_add_and_gather_match_oracle(kind, W, limit_frac, off):
    rng = np.random.default_rng(W * 13 + len(kind) + int((limit_frac or 0) * 100))
    n_op, n_cache = 300, 400
    idx = _index(rng, kind, n_op, n_cache - off[1])
    limit = None if limit_frac is None else int((n_op + off[0]) * W * limit_frac) + 3
    x = rng.standard_normal((n_op + off[0]) * W).astype(np.float32)
    y = rng.standard_normal(n_cache * W).astype(np.float32)
    e = y.copy()
    oracle.add_rows_from_double_index(e, x, idx, off, W, limit)
    rowops.add_rows_from_double_index_cpu(y, x, idx, off, W, limit)
    assert np.array_equal(bits(y), bits(e))
    # the gather (Read of a host-tier op): cache rows -> op buffer, guard on the op buffer
    if kind != "repeated":
        cache = rng.standard_normal(n_cache * W).astype(np.float32)
        gidx = np.stack([idx[:, 0], idx[:, 1]], 1).astype(np.int64)
        gy = np.zeros((n_op + off[0]) * W, np.float32)
        ge = gy.copy()
        goff = (off[0], off[1])
        oracle.assign_rows_to_double_index(ge, cache, gidx, goff, W, limit)
        rowops.assign_rows_to_double_index_cpu(gy, cache, gidx, goff, W, limit)
        assert np.array_equal(bits(gy), bits(ge))


@pytest.mark.parametrize("kind", ["permuted", "repeated"])
def test_host_row_ops_multithreaded_keep_op_order(kind):
    """Calls of 4 MiB of rows and more run on several threads, each owning a
    range of destination rows and walking the index in order: a destination
    listed many times still gets its adds in op order, bit for bit."""
    rng = np.random.default_rng(99 + len(kind))
    W, n_op, n_cache = 128, 40000, 50000
    idx = _index(rng, kind, n_op, n_cache)
    if kind == "repeated":
        idx[::7, 1] = 123  # one row listed ~5,700 times
    x = rng.standard_normal(n_op * W).astype(np.float32)
    y = rng.standard_normal(n_cache * W).astype(np.float32)
    e = y.copy()
    oracle.add_rows_from_double_index(e, x, idx, (0, 0), W, n_op * W - 77)
    rowops.add_rows_from_double_index_cpu(y, x, idx, (0, 0), W, n_op * W - 77)
    assert np.array_equal(bits(y), bits(e))
    if kind == "permuted":
        g, ge = np.zeros(n_op * W, np.float32), np.zeros(n_op * W, np.float32)
        gidx = np.stack([np.arange(n_op), rng.integers(0, n_cache, n_op)], 1).astype(np.int64)
        oracle.assign_rows_to_double_index(ge, y, gidx, (0, 0), W, n_op * W - 5)
        rowops.assign_rows_to_double_index_cpu(g, y, gidx, (0, 0), W, n_op * W - 5)
        assert np.array_equal(bits(g), bits(ge))


def test_host_add_matches_vsadd():
    rng = np.random.default_rng(3)
    for n in (1, 127, 128 * 1000 + 5, (8 << 20) + 3):
        y = rng.standard_normal(n).astype(np.float32)
        x = rng.standard_normal(n).astype(np.float32)
        e = oracle.vs_add(y, x)
        rowops.add_row_batch_cpu(y, x)
        assert np.array_equal(bits(y), bits(e))
    empty = np.zeros(0, np.float32)
    rowops.add_row_batch_cpu(empty, empty)  # a no-op (vsAdd's n > 0 precondition does not apply)


def test_host_zero():
    from geeps_amd import native
    for n in (1, 1000, (8 << 20) + 5):
        y = np.full(n, np.float32(-3.5))
        native.check(native.lib().gp_host_zero(n - 1, y.ctypes.data), "gp_host_zero")
        assert not y[:n - 1].any() and y[n - 1] == np.float32(-3.5)
    assert native.lib().gp_host_zero(3, None) == 1


def test_host_row_ops_reject_bad_arguments_and_skip_empty_calls():
    from geeps_amd import native
    L = native.lib()
    assert L.gp_host_scatter_add_rows(None, None, None, 0, native.DoubleIndex(0, 0), 128, 10) == 0
    assert L.gp_host_scatter_add_rows(None, None, None, 3, native.DoubleIndex(0, 0), 128, 10) == 1
    assert b"gp_host_scatter_add_rows" in L.gp_last_error()
    y = np.zeros(8, np.float32)
    assert L.gp_host_gather_rows(y.ctypes.data, y.ctypes.data, y.ctypes.data, 1, native.DoubleIndex(0, 0), 0,
                                 10) == 1
    assert L.gp_host_add(4, None, None) == 1
    with pytest.raises(ValueError):
        rowops.add_rows_from_double_index_cpu(y, y.astype(np.float64), np.zeros((1, 2), np.int64))


@pytest.mark.parametrize("op", ["add", "init", "gather"])
def test_host_row_ops_refuse_rows_outside_the_arrays(op):
    """the host wrappers check every touched row against
    the numpy arrays before the C-ABI call (which trusts its pointers), as the
    device wrappers do; rows wholly past num_vals_limit on the guarded side are
    skipped, not refused."""
    fn = {"add": rowops.add_rows_from_double_index_cpu, "init": rowops.init_rows_from_double_index_cpu,
          "gather": rowops.assign_rows_to_double_index_cpu}[op]
    W = 4
    x = np.ones(3 * W, np.float32)
    y = np.zeros(5 * W, np.float32)
    # (source side, destination side) of an entry: add / init read x[id0] and
    # write y[id1]; the gather writes y[id0] from x[id1]
    def entry(src, dst):
        return np.array([[dst, src]] if op == "gather" else [[src, dst]], np.int64)
    fn(y, x, entry(2, 4), row_size=W)                      # in range
    for src, dst in ((3, 0), (0, 5), (0, 1 << 62)):
        with pytest.raises(ValueError, match="out of range"):
            fn(y, x, entry(src, dst), row_size=W)
    with pytest.raises(ValueError, match="negative"):
        fn(y, x, entry(-1, 0), row_size=W)
    with pytest.raises(ValueError, match="out of range"):  # a wrapped negative offset
        fn(y, x, entry(0, 0), index_offset=(0, -1), row_size=W)
    with pytest.raises(ValueError, match="out of range"):
        fn(y, x, entry(0, 0), index_offset=(3, 0) if op != "gather" else (0, 3), row_size=W)
    # the guarded side's rows past the limit are skipped (the reference's
    # guard), so an out-of-range row there is no error ...
    guarded_big = entry(7, 0) if op != "gather" else entry(0, 7)
    fn(y, x, guarded_big, row_size=W, num_vals_limit=3 * W)
    # ... but a row the limit lets in is checked
    with pytest.raises(ValueError, match="out of range"):
        fn(y, x, guarded_big, row_size=W, num_vals_limit=8 * W)
    # an unsigned index (the reference's size_t ids) is checked the same way,
    # including ids past 2^63 that a signed view would read as negative
    fn(y, x, entry(2, 4).astype(np.uint64), row_size=W)
    huge = entry(0, 0).astype(np.uint64)
    huge[0, 1 if op != "gather" else 0] = np.uint64(1 << 63)
    with pytest.raises(ValueError, match="out of range"):
        fn(y, x, huge, row_size=W)
    # the two in-range calls ran (the add twice), nothing else touched y
    assert np.array_equal(y[4 * W:], np.full(W, 2.0 if op == "add" else 1.0, np.float32))
    assert not y[:4 * W].any()


def test_host_row_ops_from_concurrent_callers():
    """The helper threads are one persistent pool shared by every caller
    (libgeeps' app thread and its reader threads call these at once): 6
    threads, each running large scatter-adds on its own rows, all bit-exact."""
    import threading
    rng = np.random.default_rng(7)
    W, n_op, n_cache = 128, 20000, 24000
    cases = []
    for _ in range(6):
        idx = _index(rng, "permuted", n_op, n_cache)
        x = rng.standard_normal(n_op * W).astype(np.float32)
        y = rng.standard_normal(n_cache * W).astype(np.float32)
        e = y.copy()
        oracle.add_rows_from_double_index(e, x, idx, (0, 0), W, n_op * W)
        cases.append((idx, x, y, e))
    errors = []

    def run(c):
        idx, x, y, e = c
        try:
            for _ in range(3):
                y0 = y.copy()
                rowops.add_rows_from_double_index_cpu(y0, x, idx, (0, 0), W, n_op * W)
                assert np.array_equal(bits(y0), bits(e))
        except Exception as ex:  # noqa: BLE001 (reported below)
            errors.append(ex)
    ts = [threading.Thread(target=run, args=(c,)) for c in cases]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not errors and not any(t.is_alive() for t in ts)


def test_host_row_ops_after_fork():
    """A forked child (the pool's threads are not copied into it) starts a
    pool of its own instead of waiting on the parent's workers."""
    import os
    n = (8 << 20) + 3
    y = np.ones(n, np.float32)
    rowops.add_row_batch_cpu(y, np.ones(n, np.float32))  # the parent's pool is up
    pid = os.fork()
    if pid == 0:
        code = 1
        try:
            z = np.ones(n, np.float32)
            rowops.add_row_batch_cpu(z, np.ones(n, np.float32))
            code = 0 if (z == 2).all() else 2
        finally:
            os._exit(code)
    _, status = os.waitpid(pid, 0)
    assert os.WIFEXITED(status) and os.WEXITSTATUS(status) == 0
    assert (y == 2).all()


@pytest.mark.parametrize("W,limit_frac,off", [(128, 1.0, (0, 0)), (128, 0.61, (0, 0)), (33, 0.5, (2, 3)),
                                              (1024, 0.93, (0, 0))])
@pytest.mark.parametrize("threaded", [False, True])
@pytest.mark.parametrize("kind", ["permuted", "repeated", "sparse"])
def test_host_init_is_zerofy_then_add(W, limit_frac, off, threaded, kind):
    """gp_host_scatter_init_rows (ABI 15), the host tier's fused oplog init:
    bit for bit the oracle's zerofy of the destination rows then its add,
    -0.0 deltas included (0.0f + -0.0f = +0.0f), and rows wholly or partly
    past num_vals_limit zero where the add contributed nothing."""
    rng = np.random.default_rng(11 + W)
    n_op = (40000 if threaded else 300) if W <= 128 else (5000 if threaded else 40)
    n_cache = n_op + 17
    idx = _index(rng, "permuted" if kind == "sparse" else kind, n_op, n_cache)[:n_op].copy()
    if kind == "repeated":
        idx[::7, 1] = idx[0, 1]  # one destination listed n_op / 7 times: init, then adds in entry order
    if kind == "sparse":
        idx[:, 1] *= 64  # destinations 64 rows apart: the per-thread set, not the bitmap
        n_cache = int(idx[:, 1].max()) + 1
    x = rng.standard_normal((n_op + off[0]) * W).astype(np.float32)
    x[::5] = np.float32(-0.0)
    limit = int(len(x) * limit_frac)
    y = np.full((n_cache + off[1]) * W, np.float32(7.25))
    e = y.copy()
    rows = np.unique(idx[:, 1]) + off[1]
    for r in rows:
        e[r * W:(r + 1) * W] = 0.0
    oracle.add_rows_from_double_index(e, x, idx, off, W, limit)
    rowops.init_rows_from_double_index_cpu(y, x, idx, off, W, limit)
    assert np.array_equal(bits(y), bits(e))


def test_host_pool_under_thread_sanitizer():
    """tests/apps/host_pool_stress.cpp, built with -fsanitize=thread by
    __graft_entry__.build(): 6 threads run large scatter-adds, fused inits,
    gathers, adds and zeroes through the shared worker pool, every element
    checked against a serial loop; ThreadSanitizer reports no race."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "build", "tests",
                       "host_pool_stress_tsan")
    if not os.path.exists(exe):
        pytest.skip("build() first (build/tests/host_pool_stress_tsan)")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, GP_HOST_THREADS="8", TSAN_OPTIONS="halt_on_error=1"))
    assert r.returncode == 0 and r.stdout.strip() == "ok", (r.stdout[-2000:], r.stderr[-4000:])
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-4000:]
