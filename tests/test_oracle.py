"""CPU oracle: hand-computed known answers, an independent numpy restatement,
and the committed golden fixtures (no GPU)."""
import numpy as np
import pytest

from oracle import oracle


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


# ---- known answers, computed by hand from the reference loops ----------------

def test_kat_add_rows_reversed_double_scatter():
    # 4 cache rows x 2 values; op buffer of 4 rows scattered in reverse
    # (row-op-util.hpp:121-139: y[id1] += x[id0]).
    W = 2
    y = np.array([0, 0, 1, 1, 2, 2, 3, 3], dtype=np.float32)
    x = np.array([10, 11, 20, 21, 30, 31, 40, 41], dtype=np.float32)
    idx = np.array([[0, 3], [1, 2], [2, 1], [3, 0]], dtype=np.uint64)
    oracle.add_rows_from_double_index(y, x, idx, (0, 0), W)
    assert y.tolist() == [40, 41, 31, 32, 22, 23, 13, 14]
    # applied twice accumulates
    oracle.add_rows_from_double_index(y, x, idx, (0, 0), W)
    assert y.tolist() == [80, 82, 61, 63, 42, 44, 23, 25]


def test_kat_add_rows_repeated_destination_sums_in_op_order():
    # The reference's channel check admits an op whose cache rows are {0, 0, 2}
    # (range 3 == count 3, clientlib-viter.cpp:869-873).  Its CPU twin adds the
    # repeats one after the other in op order (row-op-util.hpp:121-139); the row
    # plans' repeat layers reproduce exactly this (tests/test_gpu_parity.py::
    # test_row_plan_repeated_destinations).  fp32 order matters: 1e8 + 1 - 1e8.
    W = 1
    y = np.array([1e8, 7, 0], dtype=np.float32)
    x = np.array([1, -1e8, 5], dtype=np.float32)
    idx = np.array([[0, 0], [1, 0], [2, 2]], dtype=np.uint64)
    oracle.add_rows_from_double_index(y, x, idx, (0, 0), W)
    assert y.tolist() == [np.float32(np.float32(1e8) + 1) - np.float32(1e8), 7, 5]
    assert y[0] == 0.0  # (1e8 + 1) rounds to 1e8 in fp32; the other order would give 1
    # a gather listing a destination twice: the last assignment wins
    g = np.zeros(2, dtype=np.float32)
    oracle.assign_rows_to_double_index(g, np.array([3, 4, 5], dtype=np.float32),
                                       np.array([[0, 0], [1, 1], [0, 2]], dtype=np.uint64), (0, 0), W)
    assert g.tolist() == [5, 4]


def test_kat_add_rows_offset_and_limit():
    # offset.id0 = 1 shifts the source, offset.id1 = 2 shifts the destination;
    # num_vals_limit = 5 guards the SOURCE element index (x_idx < 5).
    W = 2
    y = np.zeros(10, dtype=np.float32)
    x = np.arange(1, 9, dtype=np.float32)          # 4 rows: [1,2][3,4][5,6][7,8]
    idx = np.array([[0, 0], [1, 1], [2, 2]], dtype=np.uint64)
    oracle.add_rows_from_double_index(y, x, idx, (1, 2), W, num_vals_limit=5)
    # r0: from row 1 (x_idx 2,3 ok) -> y row 2; r1: from row 2 (x_idx 4 ok, 5 no) -> y row 3;
    # r2: from row 3 (x_idx 6,7 >= 5) skipped.
    assert y.tolist() == [0, 0, 0, 0, 3, 4, 5, 0, 0, 0]


def test_kat_assign_to_guards_destination():
    W = 2
    x = np.arange(1, 9, dtype=np.float32)          # cache rows [1,2][3,4][5,6][7,8]
    y = np.full(6, -1, dtype=np.float32)
    idx = np.array([[0, 3], [1, 0], [2, 1]], dtype=np.uint64)  # y[id0] = x[id1]
    oracle.assign_rows_to_double_index(y, x, idx, (0, 0), W, num_vals_limit=3)
    assert y.tolist() == [7, 8, 1, -1, -1, -1]


def test_kat_assign_from():
    W = 1
    x = np.array([5, 6, 7], dtype=np.float32)
    y = np.zeros(3, dtype=np.float32)
    idx = np.array([[0, 2], [1, 0], [2, 1]], dtype=np.uint64)  # y[id1] = x[id0]
    oracle.assign_rows_from_double_index(y, x, idx, (0, 0), W)
    assert y.tolist() == [6, 7, 5]


def test_kat_apply_updates_order():
    # (((m + a) + b) + c) in fp32: the order is observable.
    m = np.array([1.0], dtype=np.float32)
    a = np.array([1e8], dtype=np.float32)
    b = np.array([-1e8], dtype=np.float32)
    c = np.array([0.5], dtype=np.float32)
    oracle.apply_updates(m, [a, b, c])
    assert m[0] == np.float32(0.5)         # 1 + 1e8 rounds to 1e8
    m2 = np.array([1.0], dtype=np.float32)
    oracle.apply_updates(m2, [b, a, c])
    assert m2[0] == np.float32(0.5)
    m3 = np.array([1.0], dtype=np.float32)
    oracle.apply_updates(m3, [c, a, b])
    assert m3[0] == np.float32(0.0)        # 1.5 + 1e8 - 1e8


def test_vs_add_rejects_nonpositive_n():
    # cpu_add CHECK_GT(n, 0) (mkl_alternate.hpp:62) aborts; the restatement errors.
    with pytest.raises(ValueError):
        oracle.vs_add(np.zeros(0, np.float32), np.zeros(0, np.float32))


def test_server_partition_matches_reference_formula():
    for R, S in [(10, 3), (8, 8), (7, 8), (1_048_576, 8), (1000, 7), (0, 4)]:
        starts, counts = oracle.server_partition(R, S)
        div, res = divmod(R, S)
        assert starts.tolist() == [div * i + min(i, res) for i in range(S)]
        assert counts.tolist() == [div + (i < res) for i in range(S)]
        assert int(counts.sum()) == R
    from geeps_amd.shard import server_partition
    for R, S in [(10, 3), (7, 8), (1000, 7)]:
        s, c = server_partition(R, S)
        so, co = oracle.server_partition(R, S)
        assert s == so.tolist() and c == co.tolist()


# ---- independent numpy restatement --------------------------------------------

def _np_rowop(kind, y, x, idx, off, W, limit):
    y = y.copy()
    for r in range(idx.shape[0]):
        if kind == "assign_to":
            src, dst, g = int(idx[r, 1]) + off[1], int(idx[r, 0]) + off[0], None
            g = dst
        else:
            src, dst = int(idx[r, 0]) + off[0], int(idx[r, 1]) + off[1]
            g = src
        for v in range(W):
            if limit is not None and g * W + v >= limit:
                continue
            if kind == "add_from":
                y[dst * W + v] = np.float32(y[dst * W + v] + x[src * W + v])
            else:
                y[dst * W + v] = x[src * W + v]
    return y


@pytest.mark.parametrize("kind", ["add_from", "assign_to", "assign_from"])
@pytest.mark.parametrize("W,limit", [(5, None), (4, 37), (8, None)])
def test_oracle_matches_numpy_restatement(kind, W, limit):
    rng = np.random.default_rng(42)
    n_cache, n_op = 40, 17
    idx = np.stack([np.arange(n_op), rng.choice(n_cache, n_op, replace=False)], 1).astype(np.uint64)
    big = max(n_cache, n_op) * W
    x = rng.random(big, dtype=np.float32)
    y = rng.random(big, dtype=np.float32)
    fn = {"add_from": oracle.add_rows_from_double_index,
          "assign_to": oracle.assign_rows_to_double_index,
          "assign_from": oracle.assign_rows_from_double_index}[kind]
    got = y.copy()
    fn(got, x, idx, (0, 0), W, limit)
    assert np.array_equal(bits(got), bits(_np_rowop(kind, y, x, idx, (0, 0), W, limit)))


def test_apply_updates_matches_numpy_sequential():
    n = 4099
    ups = [oracle.synthetic_delta(c, n) for c in range(5)]
    m = np.linspace(-1, 1, n, dtype=np.float32)
    ref = m.copy()
    for u in ups:
        ref = (ref + u).astype(np.float32)
    oracle.apply_updates(m, ups)
    assert np.array_equal(bits(m), bits(ref))


@pytest.mark.parametrize("threads", [2, 3, 8])
def test_apply_updates_mt_bit_exact(threads):
    n = 100_003
    ups = [oracle.synthetic_delta(c, n) for c in range(8)]
    a = np.zeros(n, np.float32)
    b = np.zeros(n, np.float32)
    oracle.apply_updates(a, ups)
    oracle.apply_updates(b, ups, threads=threads)
    assert np.array_equal(bits(a), bits(b))


# ---- golden fixtures -----------------------------------------------------------

def test_golden_rowops_reproduce(golden_rowops, manifest):
    fns = {"add_from": oracle.add_rows_from_double_index,
           "assign_to": oracle.assign_rows_to_double_index,
           "assign_from": oracle.assign_rows_from_double_index}
    assert manifest["rowops"], "empty manifest"
    for name, spec in manifest["rowops"].items():
        y = golden_rowops[f"{name}.y"].copy()
        fns[spec["kind"]](y, golden_rowops[f"{name}.x"], golden_rowops[f"{name}.index"],
                          tuple(spec["offset"]), spec["row_size"], spec["num_vals_limit"])
        assert np.array_equal(bits(y), bits(golden_rowops[f"{name}.expect"])), name


def test_golden_bucket_reproduce(golden_bucket):
    d = golden_bucket["deltas"]
    for c in range(d.shape[0]):
        assert np.array_equal(bits(d[c]), bits(oracle.synthetic_delta(c, d.shape[1])))
    for N in (1, 2, 8):
        m = np.zeros(d.shape[1], np.float32)
        oracle.apply_updates(m, [d[c] for c in range(N)])
        assert np.array_equal(bits(m), bits(golden_bucket[f"master_zero_N{N}"]))
    m = golden_bucket["master_seeded_init"].copy()
    oracle.apply_updates(m, [d[c] for c in range(8)])
    assert np.array_equal(bits(m), bits(golden_bucket["master_seeded_N8"]))
    # arrival order matters at the bit level: reversed order is a different vector
    assert not np.array_equal(bits(golden_bucket["master_zero_N8"]),
                              bits(golden_bucket["master_zero_N8_reversed"]))


def test_golden_manifest_hashes(golden_rowops, golden_bucket, manifest):
    import hashlib
    for key, h in manifest["sha256"].items():
        src, name = key.split(":", 1)
        arr = (golden_rowops if src == "rowops" else golden_bucket)[name]
        assert hashlib.sha256(np.ascontiguousarray(arr).tobytes()).hexdigest() == h, key
