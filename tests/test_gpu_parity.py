"""HIP path vs the CPU oracle, through the C-ABI (GPU box only).

Bar: bit-exact.  Every kernel here is integer indexing plus fp32 adds in the
reference's order, so results must match the oracle bit for bit (compared as
uint32 views, so -0.0 / NaN payloads count too).
"""
import os

import numpy as np
import pytest
import torch

from oracle import oracle

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def T(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _ops():
    from geeps_amd import rowops
    return {"add_from": (rowops.add_rows_from_double_index_gpu, oracle.add_rows_from_double_index),
            "assign_to": (rowops.assign_rows_to_double_index_gpu, oracle.assign_rows_to_double_index),
            "assign_from": (rowops.assign_rows_from_double_index_gpu,
                            oracle.assign_rows_from_double_index)}


# ---- golden fixtures -------------------------------------------------------------

def test_golden_rowops(dev, golden_rowops, manifest):
    ops = _ops()
    for name, spec in manifest["rowops"].items():
        x, y, idx = (golden_rowops[f"{name}.{k}"] for k in ("x", "y", "index"))
        ty = T(y, dev)
        ops[spec["kind"]][0](ty, T(x, dev), T(idx, dev), idx.shape[0], tuple(spec["offset"]),
                             spec["row_size"], spec["num_vals_limit"])
        torch.cuda.synchronize()
        assert np.array_equal(bits(ty.cpu().numpy()), bits(golden_rowops[f"{name}.expect"])), name


def test_golden_bucket(dev, golden_bucket):
    from geeps_amd import rowops
    d = golden_bucket["deltas"]
    for N in (1, 2, 8):
        m = torch.zeros(d.shape[1], dtype=torch.float32, device=dev)
        rowops.apply_updates(m, [T(d[c], dev) for c in range(N)])
        torch.cuda.synchronize()
        assert np.array_equal(bits(m.cpu().numpy()), bits(golden_bucket[f"master_zero_N{N}"])), N
    m = T(golden_bucket["master_seeded_init"], dev)
    rowops.apply_updates(m, [T(d[c], dev) for c in range(8)])
    assert np.array_equal(bits(m.cpu().numpy()), bits(golden_bucket["master_seeded_N8"]))
    m = torch.zeros(d.shape[1], dtype=torch.float32, device=dev)
    rowops.apply_updates(m, [T(d[c], dev) for c in reversed(range(8))])
    assert np.array_equal(bits(m.cpu().numpy()), bits(golden_bucket["master_zero_N8_reversed"]))


# ---- randomized sweeps vs the oracle ---------------------------------------------

@pytest.mark.parametrize("kind", ["add_from", "assign_to", "assign_from"])
@pytest.mark.parametrize("W", [1, 2, 3, 4, 5, 8, 12, 16, 60, 64, 100, 128, 256, 1000, 1024, 4096])
def test_rowop_sweep(dev, kind, W):
    rng = np.random.default_rng(W * 7 + len(kind))
    n_cache = max(8, 300000 // (W * 4)) + 5
    n_op = max(1, (n_cache * 2) // 3)
    idx = np.stack([rng.permutation(n_op), rng.choice(n_cache, n_op, replace=False)], 1)
    idx = idx.astype(np.int64)
    if kind == "assign_to":
        x = rng.standard_normal(n_cache * W).astype(np.float32)
        y = rng.standard_normal(n_op * W).astype(np.float32)
    else:
        x = rng.standard_normal(n_op * W).astype(np.float32)
        y = rng.standard_normal(n_cache * W).astype(np.float32)
    for limit in (None, int(n_op * W * 0.6) + 1):
        gpu_fn, ora_fn = _ops()[kind]
        e = y.copy()
        ora_fn(e, x, idx, (0, 0), W, limit)
        ty = T(y, dev)
        gpu_fn(ty, T(x, dev), T(idx, dev), n_op, (0, 0), W, limit)
        torch.cuda.synchronize()
        assert np.array_equal(bits(ty.cpu().numpy()), bits(e)), (kind, W, limit)


@pytest.mark.parametrize("kind", ["add_from", "assign_to", "assign_from"])
def test_rowop_offsets_and_unaligned_base(dev, kind):
    """Non-zero offsets, and base pointers 4 B off 16-B alignment (scalar path)."""
    rng = np.random.default_rng(3)
    W, n_cache, n_op, off = 128, 500, 200, (13, 29)
    idx = np.stack([np.arange(n_op), rng.choice(n_cache - off[1], n_op, replace=False)], 1)
    idx = idx.astype(np.int64)
    xs = (n_cache if kind == "assign_to" else n_op + off[0]) * W
    ys = (n_op + off[0] if kind == "assign_to" else n_cache) * W
    x = rng.standard_normal(xs + 1).astype(np.float32)
    y = rng.standard_normal(ys + 1).astype(np.float32)
    gpu_fn, ora_fn = _ops()[kind]
    for shift in (0, 1):
        e = y[shift:shift + ys].copy()
        ora_fn(e, x[shift:shift + xs].copy(), idx, off, W)
        ty_full = T(y, dev)
        tx_full = T(x, dev)
        ty = ty_full[shift:shift + ys]
        gpu_fn(ty, tx_full[shift:shift + xs], T(idx, dev), n_op, off, W)
        torch.cuda.synchronize()
        assert np.array_equal(bits(ty.cpu().numpy()), bits(e)), shift
        # nothing outside the view was touched
        assert np.array_equal(bits(ty_full.cpu().numpy()[:shift]), bits(y[:shift]))


@pytest.mark.parametrize("N", list(range(1, 21)))
def test_bucket_sum_n_way(dev, N):
    """1..20 buckets (more than 8 = chained launches, order preserved)."""
    from geeps_amd import rowops
    n = 12345 + N  # ragged: not a multiple of 4
    ups = [oracle.synthetic_delta(c, n) for c in range(N)]
    m0 = np.random.default_rng(N).standard_normal(n).astype(np.float32)
    e = m0.copy()
    oracle.apply_updates(e, ups)
    m = T(m0, dev)
    rowops.bucket_sum_apply(m, [T(u, dev) for u in ups])
    torch.cuda.synchronize()
    assert np.array_equal(bits(m.cpu().numpy()), bits(e))


@pytest.mark.parametrize("N", [0, 1, 3, 8, 9, 17])
def test_bucket_sum_into_leaves_master(dev, N):
    """Out-of-place sum (the tablet server's next shard version): `out` equals the
    in-place result bit for bit, `master` is untouched, chained launches past 8."""
    from geeps_amd import rowops
    n = 40961 + N
    ups = [oracle.synthetic_delta(100 + c, n) for c in range(N)]
    m0 = np.random.default_rng(7 + N).standard_normal(n).astype(np.float32)
    e = m0.copy()
    oracle.apply_updates(e, ups)
    m = T(m0, dev)
    out = torch.full((n,), float("nan"), dtype=torch.float32, device=dev)
    rowops.bucket_sum_into(out, m, [T(u, dev) for u in ups])
    torch.cuda.synchronize()
    assert np.array_equal(bits(out.cpu().numpy()), bits(e))
    assert np.array_equal(bits(m.cpu().numpy()), bits(m0))


@pytest.mark.parametrize("n,shift", [(3 * 96 * (1 << 18) + 5, 0), (5 * 64 * (1 << 18) + 3, 1), (1 << 20, 2)])
def test_bucket_sum_into_zero_buckets_copies(dev, n, shift):
    """gp_bucket_sum_into with no buckets is a copy (libgeeps' read-my-writes
    refresh of a shard with no pending own updates): through the sweep
    kernels' copy form, whole chunks, the tile-major rest and the scalar tail,
    on 16-B-aligned and unaligned (shifted) buffers; every bit equal, `in`
    untouched."""
    from geeps_amd import rowops
    g = torch.Generator(device=dev)
    g.manual_seed(n)
    src = torch.rand(n + shift, generator=g, device=dev) - 0.5
    dst = torch.full((n + shift,), float("nan"), dtype=torch.float32, device=dev)
    s0 = src.clone()
    rowops.bucket_sum_into(dst[shift:], src[shift:], [])
    torch.cuda.synchronize()
    assert torch.equal(dst[shift:].view(torch.int32), src[shift:].view(torch.int32))
    assert torch.equal(src.view(torch.int32), s0.view(torch.int32))


@pytest.mark.parametrize("N,out_of_place", [(1, False), (3, False), (8, False), (8, True), (11, True)])
def test_bucket_sum_phase_separated_path(dev, N, out_of_place):
    """128-MiB shards take the phase-separated kernel in balanced chunks (reads
    summed into LDS and registers per chunk, then written) over their whole
    16-KiB tiles: 2 chunks of 17 tiles per block at 1 and 3 buckets, 3 of 11
    at 8 (11 buckets: a pass of 8, then one of 3).  The rest goes to the
    mixed form (one dwordx4) and the scalar form (3 floats): every element
    checked bit for bit."""
    from geeps_amd import rowops
    n = (32 << 20) + 1024 * 4 * 3 + 7
    ups = [oracle.synthetic_delta(300 + c, n) for c in range(N)]
    m0 = np.random.default_rng(N).standard_normal(n).astype(np.float32)
    e = m0.copy()
    oracle.apply_updates(e, ups)
    m = T(m0, dev)
    tb = [T(u, dev) for u in ups]
    if out_of_place:
        out = torch.full((n,), float("nan"), dtype=torch.float32, device=dev)
        rowops.bucket_sum_into(out, m, tb)
        torch.cuda.synchronize()
        assert np.array_equal(bits(m.cpu().numpy()), bits(m0))
    else:
        rowops.bucket_sum_apply(m, tb)
        out = m
    torch.cuda.synchronize()
    assert np.array_equal(bits(out.cpu().numpy()), bits(e))


@pytest.fixture(scope="module")
def large_deltas():
    """8 client buckets of 100 Mi + 20,483 floats (400 MiB each), made once."""
    n = (100 << 20) + 1024 * 4 * 5 + 3
    return n, [oracle.synthetic_delta(500 + c, n) for c in range(8)]


@pytest.mark.parametrize("N,out_of_place", [(1, False), (2, True), (3, False), (4, False),
                                            (5, True), (6, True), (8, False), (8, True)])
def test_bucket_sum_register_tiles_path(dev, large_deltas, N, out_of_place):
    """400-MiB shards: 4 whole 96-MiB sweep chunks (7 register tiles of 32
    KiB beside 160 KiB of LDS per block; 14 of 16 KiB at 1 bucket), then the
    16-MiB rest in one balanced tile-major chunk,
    one dwordx4 for the mixed form and a 3-float scalar tail: every element
    checked bit for bit, and the plan the library reports is that form."""
    import ctypes
    from geeps_amd import native, rowops
    n, allups = large_deltas
    launches, rt = ctypes.c_int(0), ctypes.c_int(0)
    native.check(native.lib().gp_bucket_sum_plan(n, N, ctypes.byref(launches), ctypes.byref(rt)))
    assert rt.value == (14 if N == 1 else 7) and launches.value >= 3
    sw = ctypes.c_int(-1)
    native.check(native.lib().gp_bucket_sum_sweep_plan(n, N, ctypes.byref(launches),
                                                        ctypes.byref(rt), ctypes.byref(sw)))
    assert (sw.value, launches.value) == (4, 5)
    ups = allups[:N]
    m0 = np.random.default_rng(N).standard_normal(n).astype(np.float32)
    e = m0.copy()
    oracle.apply_updates(e, ups)
    m = T(m0, dev)
    tb = [T(u, dev) for u in ups]
    if out_of_place:
        out = torch.full((n,), float("nan"), dtype=torch.float32, device=dev)
        rowops.bucket_sum_into(out, m, tb)
        torch.cuda.synchronize()
        assert np.array_equal(bits(m.cpu().numpy()), bits(m0))
    else:
        rowops.bucket_sum_apply(m, tb)
        out = m
    torch.cuda.synchronize()
    assert np.array_equal(bits(out.cpu().numpy()), bits(e))
    del tb, m, out
    torch.cuda.empty_cache()


@pytest.mark.parametrize("mib,N,out_of_place", [(4, 8, False), (30, 5, True), (30, 8, False),
                                                 (100, 8, True), (100, 6, False), (30, 1, False),
                                                 (100, 2, True), (64, 3, False)])
def test_bucket_sum_balanced_small_shards(dev, large_deltas, mib, N, out_of_place):
    """Shards of 4 MiB up to 3 register-form chunks take the phased kernel in
    <= 3 balanced chunks (one launch each; 4 MiB: one tile per block), plus a
    dwordx4 and a 3-float scalar tail: bit for bit."""
    import ctypes
    from geeps_amd import native, rowops
    n = (mib << 18) + 4 + 3
    launches, rt = ctypes.c_int(0), ctypes.c_int(0)
    native.check(native.lib().gp_bucket_sum_plan(n, N, ctypes.byref(launches), ctypes.byref(rt)))
    expect_rt = 20 if N <= 2 else 12 if N <= 4 else 4
    tiles, per_chunk = mib * 64, 256 * (10 + expect_rt)
    assert rt.value == expect_rt and launches.value == -(-tiles // per_chunk) <= 3
    ups = [u[:n] for u in large_deltas[1][:N]]
    m0 = np.random.default_rng(mib + N).standard_normal(n).astype(np.float32)
    e = m0.copy()
    oracle.apply_updates(e, ups)
    m = T(m0, dev)
    tb = [T(u, dev) for u in ups]
    if out_of_place:
        out = torch.full((n,), float("nan"), dtype=torch.float32, device=dev)
        rowops.bucket_sum_into(out, m, tb)
        torch.cuda.synchronize()
        assert np.array_equal(bits(m.cpu().numpy()), bits(m0))
    else:
        rowops.bucket_sum_apply(m, tb)
        out = m
    torch.cuda.synchronize()
    assert np.array_equal(bits(out.cpu().numpy()), bits(e))


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 255, 256, 257, 1023, 1024 * 256 + 3])
def test_bucket_sum_sizes_and_alignment(dev, n):
    from geeps_amd import rowops
    ups = [oracle.synthetic_delta(c, n + 1) for c in range(3)]
    for shift in (0, 1):
        e = np.zeros(n, np.float32)
        oracle.apply_updates(e, [u[shift:shift + n].copy() for u in ups])
        backing = torch.zeros(n + 1, dtype=torch.float32, device=dev)
        m = backing[shift:shift + n]
        tb = [T(u, dev)[shift:shift + n] for u in ups]
        rowops.bucket_sum_apply(m, tb)
        torch.cuda.synchronize()
        assert np.array_equal(bits(m.cpu().numpy()), bits(e)), (n, shift)
        if shift:
            assert backing[0].item() == 0.0


def test_gpu_add_and_zero(dev):
    from geeps_amd import rowops
    n = 100_001
    a, b = oracle.synthetic_delta(1, n), oracle.synthetic_delta(2, n)
    y = torch.empty(n, dtype=torch.float32, device=dev)
    rowops.gpu_add(n, T(a, dev), T(b, dev), y)
    torch.cuda.synchronize()
    assert np.array_equal(bits(y.cpu().numpy()), bits(oracle.vs_add(a, b)))
    ty = T(a, dev)
    rowops.add_row_batch_gpu(ty, T(b, dev), n // 128, 128)
    e = a.copy()
    e[:(n // 128) * 128] = oracle.vs_add(a[:(n // 128) * 128], b[:(n // 128) * 128])
    assert np.array_equal(bits(ty.cpu().numpy()), bits(e))
    rowops.zerofy_data_gpu(ty)
    assert int(torch.count_nonzero(ty)) == 0


def test_hbm_read_probe_streams_the_buffer(dev):
    """gp_hbm_probe(READ) reads every byte and writes none of them: 1 GiB takes
    at least 1 GiB / 10 TB/s (an empty kernel body -- a dead sink lets the
    compiler drop every load -- finished in microseconds), and the probed
    buffer is unchanged (its sink is a device global of its own)."""
    from geeps_amd import native
    lib = native.lib()
    n = 1 << 28
    buf = torch.rand(n, dtype=torch.float32, device=dev)
    ref = buf.clone()
    s = torch.cuda.current_stream()
    native.check(lib.gp_hbm_probe(0, buf.data_ptr(), n, s.cuda_stream), "gp_hbm_probe")
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    native.check(lib.gp_hbm_probe(0, buf.data_ptr(), n, s.cuda_stream), "gp_hbm_probe")
    b.record(s)
    b.synchronize()
    ms = a.elapsed_time(b)
    assert ms >= n * 4 / 10e12 * 1e3, f"read probe took {ms} ms for 1 GiB: loads were dropped"
    assert torch.equal(buf, ref)


def test_empty_calls_are_noops(dev):
    from geeps_amd import rowops
    y = torch.ones(256, dtype=torch.float32, device=dev)
    idx = torch.zeros((0, 2), dtype=torch.int64, device=dev)
    rowops.add_rows_from_double_index_gpu(y, y, idx, 0)
    rowops.bucket_sum_apply(y, [])
    torch.cuda.synchronize()
    assert torch.all(y == 1)


def test_out_of_range_index_rejected_before_launch(dev):
    from geeps_amd import rowops
    y = torch.zeros(4 * 128, dtype=torch.float32, device=dev)
    x = torch.zeros(4 * 128, dtype=torch.float32, device=dev)
    idx = torch.tensor([[0, 4]], dtype=torch.int64, device=dev)
    with pytest.raises(ValueError):
        rowops.add_rows_from_double_index_gpu(y, x, idx, 1)
    with pytest.raises(ValueError):
        rowops.assign_rows_to_double_index_gpu(y, x, idx, 1)


def test_side_stream(dev):
    from geeps_amd import rowops
    n = 1 << 20
    ups = [oracle.synthetic_delta(c, n) for c in range(4)]
    e = np.zeros(n, np.float32)
    oracle.apply_updates(e, ups)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        m = torch.zeros(n, dtype=torch.float32, device=dev)
        tb = [T(u, dev) for u in ups]
        rowops.bucket_sum_apply(m, tb)   # launched on s (current stream)
    s.synchronize()
    assert np.array_equal(bits(m.cpu().numpy()), bits(e))


# ---- full BASELINE sizes: every element vs torch, sampled rows vs the oracle -------

def _sample_rows(rng, R, k=2048):
    # always include the first and last rows (grid-stride head and tail)
    return np.unique(np.concatenate([[0, R - 1], rng.choice(R, size=k, replace=False)]))


@pytest.mark.parametrize("N,out_of_place", [(3, False), (5, True), (8, False), (8, True)])
def test_bucket_sum_big_and_small_sweeps(dev, N, out_of_place):
    """528 MiB + 7 floats: 4 sweep chunks of 96 MiB, 2 of 64 MiB, a 16-MiB
    tile-major chunk, one dwordx4 of the mixed form and a 3-float scalar
    tail, as the launch plan reports; every element bit for bit against a
    plain torch fp32 reference adding the buckets in client order."""
    import ctypes
    from geeps_amd import native, rowops
    n = (132 << 20) + 7
    sp = native.SumPlan()
    native.check(native.lib().gp_bucket_sum_launch_plan(n, N, ctypes.byref(sp)))
    assert (sp.sweep_launches, sp.small_sweep_launches, sp.phased_launches, sp.other_launches) == (4, 2, 1, 2)
    g = torch.Generator(device=dev)
    g.manual_seed(528 + N)
    buckets = [torch.rand(n, generator=g, device=dev) - 0.5 for _ in range(N)]
    master = torch.rand(n, generator=g, device=dev) - 0.5
    expect = master.clone()
    for b in buckets:
        expect += b
    if out_of_place:
        m0 = master.clone()
        out = torch.full((n,), float("nan"), dtype=torch.float32, device=dev)
        rowops.bucket_sum_into(out, master, buckets)
        torch.cuda.synchronize()
        assert torch.equal(master.view(torch.int32), m0.view(torch.int32))
    else:
        rowops.bucket_sum_apply(master, buckets)
        out = master
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int32), expect.view(torch.int32))


@pytest.mark.slow
def test_full_size_8way_bucket_sum(dev):
    """1M rows x 1024 fp32, 8 clients (36 GiB resident).  Every element against a
    plain torch fp32 reference in client order, and sampled rows against the C
    oracle (per-element arithmetic is independent across elements)."""
    from geeps_amd import rowops
    R, W, N = 1 << 20, 1024, 8
    n = R * W
    g = torch.Generator(device=dev)
    buckets = []
    for c in range(N):
        g.manual_seed(1000 + c)
        buckets.append(torch.rand(n, generator=g, device=dev) - 0.5)
    g.manual_seed(77)
    master = torch.rand(n, generator=g, device=dev) - 0.5
    rows = _sample_rows(np.random.default_rng(0), R)
    ridx = torch.from_numpy(rows).to(dev)
    m0 = master.view(R, W)[ridx].cpu().numpy().ravel()
    bs = [b.view(R, W)[ridx].cpu().numpy().ravel() for b in buckets]
    # every element: a plain torch fp32 reference adding the buckets one at a
    # time in client order (elementwise IEEE adds, the same order of operations)
    expect = master.clone()
    for b in buckets:
        expect += b
    rowops.bucket_sum_apply(master, buckets)
    torch.cuda.synchronize()
    assert torch.equal(master.view(torch.int32), expect.view(torch.int32))
    del expect
    oracle.apply_updates(m0, bs)
    got = master.view(R, W)[ridx].cpu().numpy().ravel()
    assert np.array_equal(bits(got), bits(m0))


@pytest.mark.slow
def test_full_size_config1_two_clients(dev):
    """BASELINE configs[1]: 1M rows x 1024 fp32, one shard, 2 clients (16 GiB
    resident with the reference copy).  The plan is 42 launches of the sweep
    kernel's 96-MiB chunks and one tile-major launch for the 64-MiB rest;
    every element against a plain torch fp32 reference adding the 2 buckets in
    client order, and sampled rows against the C oracle."""
    import ctypes
    from geeps_amd import native, rowops
    R, W, N = 1 << 20, 1024, 2
    n = R * W
    launches, rt, sw = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_int(0)
    native.check(native.lib().gp_bucket_sum_sweep_plan(n, N, ctypes.byref(launches),
                                                        ctypes.byref(rt), ctypes.byref(sw)))
    assert (sw.value, launches.value, rt.value) == (42, 43, 7)  # 7 register tiles of 32 KiB
    g = torch.Generator(device=dev)
    buckets = []
    for c in range(N):
        g.manual_seed(1000 + c)
        buckets.append(torch.rand(n, generator=g, device=dev) - 0.5)
    g.manual_seed(78)
    master = torch.rand(n, generator=g, device=dev) - 0.5
    rows = _sample_rows(np.random.default_rng(2), R)
    ridx = torch.from_numpy(rows).to(dev)
    m0 = master.view(R, W)[ridx].cpu().numpy().ravel()
    bs = [b.view(R, W)[ridx].cpu().numpy().ravel() for b in buckets]
    expect = master.clone()
    for b in buckets:
        expect += b
    rowops.bucket_sum_apply(master, buckets)
    torch.cuda.synchronize()
    assert torch.equal(master.view(torch.int32), expect.view(torch.int32))
    del expect
    oracle.apply_updates(m0, bs)
    got = master.view(R, W)[ridx].cpu().numpy().ravel()
    assert np.array_equal(bits(got), bits(m0))


@pytest.mark.slow
def test_full_size_scatter_add_permuted(dev):
    """8M RowData rows (the 1M x 1024 table through the 128-float API), random
    permutation DoubleIndex; every row vs a torch reference and sampled rows vs
    the oracle, and x added then subtracted restores y bit-exactly on
    integer-valued data."""
    from geeps_amd import rowops
    R, W = 1 << 23, 128
    g = torch.Generator(device=dev)
    g.manual_seed(11)
    perm = torch.randperm(R, generator=g, device=dev)
    idx = torch.stack([torch.arange(R, device=dev), perm], 1).contiguous()
    x = torch.randint(-64, 64, (R * W,), generator=g, device=dev).float()
    y = torch.randint(-64, 64, (R * W,), generator=g, device=dev).float()
    y0 = y.clone()
    rows = _sample_rows(np.random.default_rng(1), R)
    rowops.add_rows_from_double_index_gpu(y, x, idx, R, (0, 0), W, R * W, validate=False)
    torch.cuda.synchronize()
    # oracle on the sampled op rows: y[perm[r]] = y0[perm[r]] + x[r]
    pr = perm.cpu().numpy()[rows]
    ridx, pidx = torch.from_numpy(rows).to(dev), torch.from_numpy(pr).to(dev)
    got = y.view(R, W)[pidx].cpu().numpy()
    e = y0.view(R, W)[pidx].cpu().numpy() + x.view(R, W)[ridx].cpu().numpy()
    assert np.array_equal(bits(got), bits(e.astype(np.float32)))
    # every row: the torch reference y0[perm[r]] + x[r] (integer-valued, exact)
    full = y0.view(R, W).clone()
    full[perm] = full[perm] + x.view(R, W)
    assert torch.equal(y.view(R, W).view(torch.int32), full.view(torch.int32))
    del full
    rowops.add_rows_from_double_index_gpu(y, -x, idx, R, (0, 0), W, R * W, validate=False)
    torch.cuda.synchronize()
    assert torch.equal(y, y0)


@pytest.mark.slow
def test_sum_past_the_reference_int_range(dev):
    """The reference's sum takes an `int` element count (cpu_add<float>, CHECK_GT
    n > 0, math_functions.cpp:132-136; CUDA_KERNEL_LOOP's int index,
    device_alternate.hpp:31-54), so one call stops short of 2^31 elements.  The
    C-ABI's counts are size_t: a 2-bucket sum over 2^31 + 4,099 floats (8 GiB
    per buffer, a ragged tail through the tile-major and scalar forms) is
    bit-exact against torch fp32 in client order over every element."""
    from geeps_amd import rowops
    n = (1 << 31) + 4099
    g = torch.Generator(device=dev)
    g.manual_seed(31)
    buckets = [torch.rand(n, generator=g, device=dev) - 0.5 for _ in range(2)]
    master = torch.rand(n, generator=g, device=dev) - 0.5
    expect = master.clone()
    for b in buckets:
        expect += b
    rowops.bucket_sum_apply(master, buckets)
    torch.cuda.synchronize()
    assert torch.equal(master.view(torch.int32), expect.view(torch.int32))


@pytest.mark.slow
def test_row_ops_past_the_reference_int_range(dev):
    """2^24 + 7 RowData rows = 2^31 + 896 floats per side, past the
    reference kernels' int element index (row-op-util.cu's CUDA_KERNEL_LOOP):
    the unplanned scatter-add on a random permutation (its first call builds
    the inverse map, the second runs it behind the device check) and the
    gather with the roles swapped, every row against torch on integer-valued
    data (exact)."""
    from geeps_amd import rowops
    R, W = (1 << 24) + 7, 128
    g = torch.Generator(device=dev)
    g.manual_seed(24)
    perm = torch.randperm(R, generator=g, device=dev)
    idx = torch.stack([torch.arange(R, device=dev), perm], 1).contiguous()
    x = torch.randint(-64, 64, (R * W,), generator=g, device=dev).float()
    y = torch.randint(-64, 64, (R * W,), generator=g, device=dev).float()
    full = y.view(R, W).clone()
    full[perm] += x.view(R, W)
    for call in range(2):  # y + x, then y + 2x
        rowops.add_rows_from_double_index_gpu(y, x, idx, R, (0, 0), W, R * W, validate=False)
        torch.cuda.synchronize()
        assert torch.equal(y.view(R, W).view(torch.int32), full.view(torch.int32)), call
        full[perm] += x.view(R, W)
    del full
    out = torch.zeros(R * W, device=dev)
    gidx = torch.stack([perm, torch.arange(R, device=dev)], 1).contiguous()  # out[perm[r]] = y[r]
    rowops.assign_rows_to_double_index_gpu(out, y, gidx, R, (0, 0), W, R * W, validate=False)
    torch.cuda.synchronize()
    assert torch.equal(out.view(R, W)[perm], y.view(R, W))


@pytest.mark.parametrize("W,limit_frac,shift", [(128, None, 0), (64, 0.55, 0), (130, None, 0),
                                               (128, 0.7, 1), (1024, None, 0)])
def test_scatter_init_equals_zero_then_add(dev, W, limit_frac, shift):
    """gp_scatter_init_rows == zerofy + add_rows_from_double_index on every listed
    destination row (the oracle: zeros, then the reference add), including -0.0
    deltas (0.0f + -0.0f = +0.0f) and rows past num_vals_limit; rows not listed
    keep their old contents."""
    from geeps_amd import rowops
    rng = np.random.default_rng(W + int((limit_frac or 0) * 100))
    n_cache, n_op = 600, 400
    dst = rng.choice(n_cache, n_op, replace=False)
    idx = np.stack([rng.permutation(n_op), dst], 1).astype(np.int64)
    x = rng.standard_normal(n_op * W + 1).astype(np.float32)
    x[rng.choice(n_op * W, 500, replace=False)] = np.float32(-0.0)
    y = rng.standard_normal(n_cache * W + 1).astype(np.float32)
    limit = None if limit_frac is None else int(n_op * W * limit_frac) + 3
    xs, ys = x[shift:shift + n_op * W].copy(), y[shift:shift + n_cache * W].copy()
    e = ys.copy()
    listed = np.zeros(n_cache, bool)
    listed[dst] = True
    e.reshape(n_cache, W)[listed] = 0.0
    oracle.add_rows_from_double_index(e, xs, idx, (0, 0), W, limit)
    ty_full, tx_full = T(y, dev), T(x, dev)
    ty = ty_full[shift:shift + n_cache * W]
    rowops.init_rows_from_double_index_gpu(ty, tx_full[shift:shift + n_op * W], T(idx, dev),
                                           n_op, (0, 0), W, limit)
    torch.cuda.synchronize()
    assert np.array_equal(bits(ty.cpu().numpy()), bits(e))


# ---- segmented param cache (libgeeps refresh slots) --------------------------------

def _split(rng, n_cache, k):
    cuts = np.sort(rng.choice(np.arange(1, n_cache), k - 1, replace=False)) if k > 1 else []
    return [0] + [int(c) for c in cuts] + [n_cache]


@pytest.mark.parametrize("W", [1, 3, 4, 64, 100, 128, 1000])
@pytest.mark.parametrize("nseg", [1, 2, 8, 64])
def test_segmented_gather_and_add(dev, W, nseg):
    """Gather from / scatter-add into a cache split over separate buffers equals
    the flat-cache oracle bit for bit (offsets, num_vals_limit tails included)."""
    from geeps_amd import rowops
    rng = np.random.default_rng(W * 131 + nseg)
    n_cache = max(nseg + 1, 200000 // (W * 4))
    n_op = max(1, n_cache // 2)
    bounds = _split(rng, n_cache, nseg)
    cache = rng.standard_normal(n_cache * W).astype(np.float32)
    # odd starting offsets: the buffers are views one float into a larger one,
    # so for W % 4 == 0 the scalar (unaligned) path runs for half the cases
    pad = 1 if (W * nseg) % 2 else 0

    def seg_tensors(c):
        out = []
        for i in range(nseg):
            a, b = bounds[i], bounds[i + 1]
            big = torch.empty((b - a) * W + pad, dtype=torch.float32, device=dev)
            t = big[pad:]
            t.copy_(T(c[a * W:b * W], dev))
            out.append((a, t))
        return out

    off1 = 3
    idx = np.stack([rng.permutation(n_op), rng.choice(n_cache - off1, n_op, replace=False)], 1)
    idx = idx.astype(np.int64)
    for limit in (None, int(n_op * W * 0.7) + 1):
        # gather: y[id0] = cache[id1 + off1]
        y = rng.standard_normal(n_op * W).astype(np.float32)
        e = y.copy()
        oracle.assign_rows_to_double_index(e, cache, idx, (0, off1), W, limit)
        ty = T(y, dev)
        rowops.gather_rows_segmented(ty, seg_tensors(cache), T(idx, dev), n_op, (0, off1), W, limit)
        torch.cuda.synchronize()
        assert np.array_equal(bits(ty.cpu().numpy()), bits(e)), ("gather", limit)
        # scatter-add: cache[id1 + off1] += x[id0]
        x = rng.standard_normal(n_op * W).astype(np.float32)
        e = cache.copy()
        oracle.add_rows_from_double_index(e, x, idx, (0, off1), W, limit)
        segs = seg_tensors(cache)
        rowops.add_rows_segmented(segs, T(x, dev), T(idx, dev), n_op, (0, off1), W, limit)
        torch.cuda.synchronize()
        got = np.concatenate([t.cpu().numpy() for _, t in segs])
        assert np.array_equal(bits(got), bits(e)), ("add", limit)


def test_segmented_rejects_bad_tables(dev):
    from geeps_amd import native, rowops
    y = torch.zeros(128 * 4, device=dev)
    c = torch.zeros(128 * 4, device=dev)
    idx = torch.tensor([[0, 0]], dtype=torch.int64, device=dev)
    with pytest.raises(ValueError):
        rowops.gather_rows_segmented(y, [(1, c)], idx)
    with pytest.raises(ValueError):
        rowops.gather_rows_segmented(y, [(0, c), (0, c)], idx)
    with pytest.raises(ValueError):
        rowops.gather_rows_segmented(y, [(0, c)] + [(i + 1, c) for i in range(64)], idx)
    # the C-ABI itself rejects them too (no host validation in between)
    t = native.RowSegments()
    t.count = 2
    t.first_row[0], t.first_row[1] = 0, 0
    t.base[0] = t.base[1] = c.data_ptr()
    rc = native.lib().gp_gather_rows_segmented(y.data_ptr(), t, idx.data_ptr(), 1,
                                               native.DoubleIndex(0, 0), 128, 1 << 40, None)
    assert rc == native.GP_ERR_INVALID
    t.count = 0
    rc = native.lib().gp_scatter_add_rows_segmented(t, y.data_ptr(), idx.data_ptr(), 1,
                                                    native.DoubleIndex(0, 0), 128, 1 << 40, None)
    assert rc == native.GP_ERR_INVALID


# ---- row plans (compiled DoubleIndex: dense runs + id1-sorted residual) ----------

def _plan_index(rng, kind, n_cache, W):
    """(index, n_op): identity; a random permutation; or a mix of 3 dense runs
    (listed out of order), short runs and scattered rows."""
    if kind == "identity":
        n = n_cache
        return np.stack([np.arange(n), np.arange(n)], 1).astype(np.int64), n
    if kind == "permuted":
        n = n_cache
        return np.stack([np.arange(n), rng.permutation(n)], 1).astype(np.int64), n
    run = max(1, (4 << 20) // (W * 4))
    dst = rng.permutation(n_cache)
    parts, j0, d0 = [], 0, 0
    for L in (run, 5, run + 3, 1, 2 * run, 17):
        parts.append(np.stack([j0 + np.arange(L), d0 + np.arange(L)], 1))
        j0, d0 = j0 + L, d0 + L + 2  # a 2-row gap between destination runs
    used = np.concatenate([p[:, 1] for p in parts])
    free = np.setdiff1d(np.arange(n_cache), used)
    k = min(len(free), 3000)
    parts.append(np.stack([j0 + np.arange(k), rng.choice(free, k, replace=False)], 1))
    idx = np.concatenate(parts)
    return idx[rng.permutation(idx.shape[0])].astype(np.int64), idx.shape[0]


def _op_order_index(rng, kind, n, W):
    """An index in op order for the unplanned calls' device plans: identity;
    a random permutation of destinations; destinations ascending with gaps and
    random sources ("sorted"); or "runs": three dense runs (>= 4 MiB each, the
    second's destinations below the first's) with scattered rows between and
    around them, all in op order."""
    if kind == "identity":
        return np.stack([np.arange(n), np.arange(n)], 1).astype(np.int64)
    if kind == "permuted":
        return np.stack([np.arange(n), rng.permutation(n)], 1).astype(np.int64)
    if kind == "sorted":
        dst = np.sort(rng.choice(n + n // 3, n, replace=False))
        return np.stack([rng.permutation(n), dst], 1).astype(np.int64)
    run = (4 << 20) // (W * 4) + 130
    assert n > 3 * run + 3000
    runs_dst = [2 * run + 50, 3, 3 * run + 500]  # destination starts, out of order
    used = np.concatenate([d + np.arange(run) for d in runs_dst])
    free = rng.permutation(np.setdiff1d(np.arange(n + 4 * run), used))
    parts, j, f = [], 0, 0
    for k, d in enumerate(runs_dst):
        m = [700, 37, 1100][k]  # scattered rows before each run
        parts.append(np.stack([j + np.arange(m), free[f:f + m]], 1))
        j, f = j + m, f + m
        parts.append(np.stack([j + np.arange(run), d + np.arange(run)], 1))
        j += run
    m = n - j
    parts.append(np.stack([j + np.arange(m), free[f:f + m]], 1))
    return np.concatenate(parts).astype(np.int64)


@pytest.fixture
def analyzed(dev):
    """Every unplanned call plans itself on the device (threshold 0), for
    this test; the default (64 MiB) afterwards."""
    from geeps_amd import native
    native.check(native.lib().gp_set_unplanned_min_bytes(0), "gp_set_unplanned_min_bytes")
    native.check(native.lib().gp_unplanned_cache_clear(), "gp_unplanned_cache_clear")
    yield
    native.check(native.lib().gp_set_unplanned_min_bytes(64 << 20), "gp_set_unplanned_min_bytes")
    native.check(native.lib().gp_unplanned_cache_clear(), "gp_unplanned_cache_clear")


def _cache_entries():
    import ctypes
    from geeps_amd import native
    e, b = ctypes.c_size_t(), ctypes.c_size_t()
    native.check(native.lib().gp_unplanned_cache_entries(ctypes.byref(e), ctypes.byref(b)),
                 "gp_unplanned_cache_entries")
    return e.value, b.value


@pytest.mark.parametrize("kind", ["identity", "permuted", "sorted", "runs"])
@pytest.mark.parametrize("W,limit_frac,off", [(128, None, (0, 0)), (64, 0.9, (5, 3)), (1024, None, (0, 2))])
def test_unplanned_device_plan_matches_oracle(analyzed, dev, kind, W, limit_frac, off):
    """The unplanned gp_scatter_add_rows / gp_scatter_init_rows /
    gp_gather_rows (the reference binding's calls) with the device-built plan:
    the index scan finds the op-order dense runs (swept), the residual is
    binned by destination (scatter-add, unsorted) or kept in order; bit for bit
    against the oracle, with offsets and num_vals_limit tails."""
    from geeps_amd import rowops
    rng = np.random.default_rng(W * 13 + len(kind))
    n = 3 * ((4 << 20) // (W * 4) + 130) + 9000
    idx = _op_order_index(rng, kind, n, W)
    n_cache = int(idx[:, 1].max()) + 1 + off[1]
    limit = None if limit_frac is None else int((n + off[0]) * W * limit_frac) + 3
    x = rng.standard_normal((n + off[0]) * W).astype(np.float32)
    x[rng.choice(x.size, 200, replace=False)] = np.float32(-0.0)
    y = rng.standard_normal(n_cache * W).astype(np.float32)
    ti = torch.from_numpy(idx).to(dev)
    tx = T(x, dev)
    # add, three times: the first call plans (an unsorted residual of rows up
    # to 128 floats: the inverse map, built and run; wider rows: op order and
    # a copy of the index, the second call then builds and runs the
    # destination-sorted residual), later calls run the plan from the cache
    e = y.copy()
    oracle.add_rows_from_double_index(e, x, idx, off, W, limit)
    for call in range(3):
        ty = T(y, dev)
        rowops.add_rows_from_double_index_gpu(ty, tx, ti, n, off, W, limit)
        torch.cuda.synchronize()
        assert np.array_equal(bits(ty.cpu().numpy()), bits(e)), ("add", kind, W, call)
    cached_add = _cache_entries()[0]
    # init: listed rows zeroed, then the add
    e = y.copy()
    e.reshape(n_cache, W)[idx[:, 1] + off[1]] = 0.0
    oracle.add_rows_from_double_index(e, x, idx, off, W, limit)
    for call in range(3):
        ty = T(y, dev)
        rowops.init_rows_from_double_index_gpu(ty, tx, ti, n, off, W, limit)
        torch.cuda.synchronize()
        assert np.array_equal(bits(ty.cpu().numpy()), bits(e)), ("init", kind, W, call)
    # every large call keeps its plan (ABI 11): an inverse map or sorted
    # residual for an unsorted residual of >= 16 MiB ("permuted" at 128 and
    # 1024 floats, "runs" at 1024), else its runs and residual ranges
    assert cached_add == 1, (kind, W)
    assert _cache_entries()[0] == 2
    # gather with the index's roles swapped: y[id0] = x[id1]
    gidx = np.ascontiguousarray(idx[:, ::-1]) if kind != "sorted" else idx
    g_out = int(gidx[:, 0].max()) + 1 + off[0]
    src = rng.standard_normal((int(gidx[:, 1].max()) + 1 + off[1]) * W).astype(np.float32)
    out = rng.standard_normal(g_out * W).astype(np.float32)
    e = out.copy()
    g_lim = None if limit is None else int(g_out * W * 0.9) + 1
    oracle.assign_rows_to_double_index(e, src, gidx, off, W, g_lim)
    to = T(out, dev)
    rowops.assign_rows_to_double_index_gpu(to, T(src, dev), torch.from_numpy(gidx).to(dev), n, off, W, g_lim)
    torch.cuda.synchronize()
    assert np.array_equal(bits(to.cpu().numpy()), bits(e)), ("gather", kind, W)


@pytest.mark.parametrize("id0", ["position", "permuted"])
def test_unplanned_plan_cache_checks_index_content(analyzed, dev, id0):
    """The plan cache keys on the index pointer but trusts no pointer: the same
    device tensor refilled with another permutation (same size, offsets,
    limit) must give the new index's sums, not the cached plan's.  The first
    call with an index builds its inverse plan (a map over destination rows)
    and runs it; later calls are steady-state calls.  The first with new
    content finds the change with its device check and only the gated
    op-order form runs (no host round trip); the next sees the check's
    host-visible word, drops the entry and plans the new index afresh
    (VERDICT r03 #4).  id0 "position" (the op buffer's rows in order, as the
    reference lists them) is checked against the compact copy (id1 only), a
    permuted id0 against the full copy."""
    from geeps_amd import native, rowops
    s0 = native.unplanned_stats()
    rng = np.random.default_rng(99)
    W, n = 128, 40000  # 20 MiB of rows: a cached (unsorted) residual
    x = rng.standard_normal(n * W).astype(np.float32)
    y = rng.standard_normal(n * W).astype(np.float32)
    tx = T(x, dev)
    ti = torch.empty((n, 2), dtype=torch.int64, device=dev)
    for round_ in range(3):
        src = np.arange(n) if id0 == "position" else rng.permutation(n)
        idx = np.stack([src, rng.permutation(n)], 1).astype(np.int64)
        if round_ == 2:  # one swapped pair: a single differing entry
            idx = prev.copy()
            idx[[5, n - 7], 1] = idx[[n - 7, 5], 1]
        ti.copy_(torch.from_numpy(idx))
        e = y.copy()
        oracle.add_rows_from_double_index(e, x, idx, (0, 0), W)
        for call in range(4 if round_ else 3):
            ty = T(y, dev)
            rowops.add_rows_from_double_index_gpu(ty, tx, ti, n, (0, 0), W)
            torch.cuda.synchronize()
            assert np.array_equal(bits(ty.cpu().numpy()), bits(e)), (round_, call)
            # one entry: the index's copy (16 B a row) and its plan: the
            # inverse map (8 B a destination row) and the compact copy (4 B)
            assert _cache_entries() == (1, 28 * n), (round_, call)
        prev = idx
    # what ran (gp_unplanned_stats_get): 3 first calls (the first sighting and
    # one re-plan per change), each building an inverse map; the other 8 calls
    # steady, 2 of which found the change and had their plan dropped by the
    # call after them
    s1 = native.unplanned_stats()
    d = {k: s1[k] - s0[k] for k in s1}
    assert d == {"scans": 3, "steady_calls": 8, "stale_drops": 2, "inverse_plans": 3, "sorted_plans": 0,
                 "ranges_plans": 0}, d


def test_unplanned_repeated_destination_marks_the_inverse_map_unsound(analyzed, dev):
    """A destination listed twice breaks the calls' precondition (the
    reference's kernel races on it, row-op-util.cu:109-125): the inverse map
    can list only one of the two entries.  inverse_count_kernel finds fewer
    listed rows than entries, the gated op-order form runs instead of the
    map's walk, and the next call drops the plan and plans afresh
    (gp_unplanned_stats_get).  The repeated entries' source rows are zero
    here, so the sums are the same whatever order the racing adds land in,
    and exact."""
    from geeps_amd import native, rowops
    rng = np.random.default_rng(17)
    W, n = 128, 40000
    idx = np.stack([np.arange(n), rng.permutation(n)], 1).astype(np.int64)
    a = rng.choice(n, 64, replace=False)
    b, c = a[:32], a[32:]
    idx[c, 1] = idx[b, 1]  # 32 destinations listed twice
    x = rng.standard_normal(n * W).astype(np.float32)
    x.reshape(n, W)[idx[a, 0]] = 0.0
    y = rng.standard_normal(n * W).astype(np.float32)
    e = y.copy()
    oracle.add_rows_from_double_index(e, x, idx, (0, 0), W)
    tx, ti = T(x, dev), torch.from_numpy(idx).to(dev)
    s0 = native.unplanned_stats()
    for call in range(2):
        ty = T(y, dev)
        rowops.add_rows_from_double_index_gpu(ty, tx, ti, n, (0, 0), W, validate=False)
        torch.cuda.synchronize()
        assert np.array_equal(bits(ty.cpu().numpy()), bits(e)), call
    s1 = native.unplanned_stats()
    d = {k: s1[k] - s0[k] for k in s1}
    assert d["inverse_plans"] == 2 and d["scans"] == 2 and d["stale_drops"] == 1 and d["steady_calls"] == 0, d


def test_unplanned_cache_capacity_bound(analyzed, dev):
    """gp_set_unplanned_cache_bytes (ABI 11): the plan cache's HBM
    is bounded by the caller.  At 0 nothing is kept (every call plans afresh,
    in op order) and the sums stay exact; the default bound afterwards caches
    again."""
    from geeps_amd import native, rowops
    rng = np.random.default_rng(11)
    W, n = 128, 40000
    x = rng.standard_normal(n * W).astype(np.float32)
    y = rng.standard_normal(n * W).astype(np.float32)
    idx = np.stack([np.arange(n), rng.permutation(n)], 1).astype(np.int64)
    tx, ti = T(x, dev), torch.from_numpy(idx).to(dev)
    e = y.copy()
    oracle.add_rows_from_double_index(e, x, idx, (0, 0), W)
    try:
        native.check(native.lib().gp_set_unplanned_cache_bytes(0), "gp_set_unplanned_cache_bytes")
        for call in range(3):
            ty = T(y, dev)
            rowops.add_rows_from_double_index_gpu(ty, tx, ti, n, (0, 0), W)
            torch.cuda.synchronize()
            assert np.array_equal(bits(ty.cpu().numpy()), bits(e)), call
            assert _cache_entries() == (0, 0), call
    finally:
        native.check(native.lib().gp_set_unplanned_cache_bytes(4 << 30), "gp_set_unplanned_cache_bytes")
    rowops.add_rows_from_double_index_gpu(T(y, dev), tx, ti, n, (0, 0), W)
    torch.cuda.synchronize()
    assert _cache_entries()[0] == 1


def test_unplanned_steady_state_does_not_wait_for_the_device(analyzed, dev):
    """once an index is planned and cached, an unplanned call
    only queues work (the device check, then both gated outcomes): it must
    return while the stream is still busy with earlier work, where the
    round-3 form copied the check's result to the host and synced first.  The
    results stay bit-exact, for an unchanged index and for one changed in
    place behind the busy stream."""
    from geeps_amd import rowops
    if not hasattr(torch.cuda, "_sleep"):
        pytest.skip("torch.cuda._sleep unavailable")
    rng = np.random.default_rng(5)
    W, n = 128, 40000
    x = rng.standard_normal(n * W).astype(np.float32)
    y = rng.standard_normal(n * W).astype(np.float32)
    idx = np.stack([np.arange(n), rng.permutation(n)], 1).astype(np.int64)
    tx, ti = T(x, dev), torch.from_numpy(idx).to(dev)
    for _ in range(3):  # first sighting, sort, steady state
        rowops.add_rows_from_double_index_gpu(T(y, dev), tx, ti, n, (0, 0), W, validate=False)
    torch.cuda.synchronize()
    for changed in (False, True):
        idx2 = idx.copy()
        if changed:
            idx2[[3, 11], 1] = idx2[[11, 3], 1]
        e = y.copy()
        oracle.add_rows_from_double_index(e, x, idx2, (0, 0), W)
        ty, ti2 = T(y, dev), torch.from_numpy(idx2).to(dev)
        torch.cuda.synchronize()
        stream = torch.cuda.current_stream()
        torch.cuda._sleep(200_000_000)  # ~0.1 s of device time ahead of the call
        ti.copy_(ti2)  # device to device, stream-ordered behind the sleep
        rowops.add_rows_from_double_index_gpu(ty, tx, ti, n, (0, 0), W, validate=False)
        busy = not stream.query()
        torch.cuda.synchronize()
        assert busy, "the steady-state call waited for the device"
        assert np.array_equal(bits(ty.cpu().numpy()), bits(e)), changed


def test_unplanned_unsound_map_stays_unsound_for_queued_calls(analyzed, dev):
    """an inverse map found unsound at its build (here a
    source row at or above 2^32, which the map's 4-B field would cut) must not
    be walked by a call queued right behind the build, before the host can
    see the finding.  The build's kernels set a sticky device word that every
    later call's index check reads.  Two calls back to back with no sync, then
    a third after one: all bit-exact against the oracle (the far source rows
    mapped to a compact host copy for it).  x spans 2^32 + 64 rows of 4 floats
    (64 GiB of HBM, mostly never touched)."""
    from geeps_amd import native, rowops
    rng = np.random.default_rng(23)
    W, n, far = 4, 4 << 20, 64
    src = np.arange(n, dtype=np.int64)
    picks = rng.choice(n, far, replace=False)
    src[picks] = (1 << 32) + np.arange(far)
    idx = np.stack([src, rng.permutation(n)], 1).astype(np.int64)
    x_near = rng.standard_normal(n * W).astype(np.float32)
    x_far = rng.standard_normal(far * W).astype(np.float32)
    y = rng.standard_normal(n * W).astype(np.float32)
    # the oracle on a compact x: far row 2^32 + j -> row n + j
    compact = idx.copy()
    compact[picks, 0] = n + np.arange(far)
    e = y.copy()
    oracle.add_rows_from_double_index(e, np.concatenate([x_near, x_far]), compact, (0, 0), W)
    tx = torch.empty(((1 << 32) + far) * W, dtype=torch.float32, device=dev)
    tx[:n * W].copy_(torch.from_numpy(x_near))
    tx[(1 << 32) * W:].copy_(torch.from_numpy(x_far))
    ti = torch.from_numpy(idx).to(dev)
    ys = [T(y, dev) for _ in range(3)]
    torch.cuda.synchronize()
    s0 = native.unplanned_stats()
    rowops.add_rows_from_double_index_gpu(ys[0], tx, ti, n, (0, 0), W, validate=False)  # builds the map
    rowops.add_rows_from_double_index_gpu(ys[1], tx, ti, n, (0, 0), W, validate=False)  # queued behind it
    torch.cuda.synchronize()
    rowops.add_rows_from_double_index_gpu(ys[2], tx, ti, n, (0, 0), W, validate=False)
    torch.cuda.synchronize()
    d = {k: v - s0[k] for k, v in native.unplanned_stats().items()}
    for call, ty in enumerate(ys):
        assert np.array_equal(bits(ty.cpu().numpy()), bits(e)), call
    assert d["inverse_plans"] >= 1, d
    del tx, ys
    torch.cuda.empty_cache()


def test_unplanned_plan_drop_does_not_wait_for_other_streams(analyzed, dev):
    """dropping a cached plan (an index refilled in place at
    the same pointer, or an eviction) retires its buffers in stream order
    behind the calls that used them; round 4 synchronised the whole device,
    stalling every other stream of the process (libgeeps' server and reader
    streams).  A call that drops a stale plan must return while another
    stream is still busy with ~0.1 s of work; results stay exact."""
    from geeps_amd import native, rowops
    if not hasattr(torch.cuda, "_sleep"):
        pytest.skip("torch.cuda._sleep unavailable")
    rng = np.random.default_rng(31)
    W, n = 128, 40000
    x = rng.standard_normal(n * W).astype(np.float32)
    y = rng.standard_normal(n * W).astype(np.float32)
    idx = np.stack([np.arange(n), rng.permutation(n)], 1).astype(np.int64)
    idx2 = idx.copy()
    idx2[[5, 17], 1] = idx2[[17, 5], 1]
    tx, ti = T(x, dev), torch.from_numpy(idx).to(dev)
    for _ in range(3):  # planned, steady
        rowops.add_rows_from_double_index_gpu(T(y, dev), tx, ti, n, (0, 0), W, validate=False)
    ti.copy_(torch.from_numpy(idx2).to(dev))  # refilled in place
    rowops.add_rows_from_double_index_gpu(T(y, dev), tx, ti, n, (0, 0), W, validate=False)  # finds the change
    torch.cuda.synchronize()
    e = y.copy()
    oracle.add_rows_from_double_index(e, x, idx2, (0, 0), W)
    ty = T(y, dev)
    side, mine = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    s0 = native.unplanned_stats()
    with torch.cuda.stream(side):
        torch.cuda._sleep(200_000_000)  # ~0.1 s on another stream
    with torch.cuda.stream(mine):
        rowops.add_rows_from_double_index_gpu(ty, tx, ti, n, (0, 0), W, validate=False)  # drops the stale plan
    busy = not side.query()
    torch.cuda.synchronize()
    d = {k: v - s0[k] for k, v in native.unplanned_stats().items()}
    assert d["stale_drops"] == 1, d
    assert busy, "dropping the stale plan waited for another stream"
    assert np.array_equal(bits(ty.cpu().numpy()), bits(e))


@pytest.mark.parametrize("kind", ["identity", "permuted", "mixed"])
@pytest.mark.parametrize("W,limit_frac,off", [(128, None, (0, 0)), (64, None, (5, 3)),
                                               (128, 0.83, (0, 0)), (1024, None, (0, 2)),
                                               (130, None, (0, 0)), (4, 0.5, (1, 1))])
def test_row_plan_matches_oracle(dev, kind, W, limit_frac, off):
    """gp_scatter_add_rows_planned / gp_scatter_init_rows_planned equal the
    oracle's add_rows_from_double_index (init: on zeroed listed rows) bit for
    bit, with the plan's dense runs, residual rows, offsets and num_vals_limit
    tails; rows not listed are untouched."""
    from geeps_amd import rowops
    rng = np.random.default_rng(W * 7 + len(kind) + int((limit_frac or 0) * 10))
    n_cache = 5 * ((4 << 20) // (W * 4)) + 8000
    idx, n_op = _plan_index(rng, kind, n_cache - off[1], W)
    limit = None if limit_frac is None else int((n_op + off[0]) * W * limit_frac) + 3
    x = rng.standard_normal((n_op + off[0]) * W).astype(np.float32)
    x[rng.choice(x.size, 300, replace=False)] = np.float32(-0.0)
    y = rng.standard_normal(n_cache * W).astype(np.float32)
    plan = rowops.RowPlan(idx, n_op, off, W, limit)
    info = plan.info()
    assert info["rows"] == n_op
    if kind == "identity" and limit is None:
        assert info == {"rows": n_op, "dense_runs": 1, "dense_rows": n_op, "residual_rows": 0,
                        "repeat_layers": 0, "repeat_rows": 0}
    if kind == "mixed" and limit is None:
        assert info["dense_runs"] == 3 and info["residual_rows"] > 0
    if kind == "permuted":
        assert info["dense_runs"] == 0
    # add
    e = y.copy()
    oracle.add_rows_from_double_index(e, x, idx, off, W, limit)
    ty = T(y, dev)
    plan.add(ty, T(x, dev))
    torch.cuda.synchronize()
    assert np.array_equal(bits(ty.cpu().numpy()), bits(e)), ("add", kind, W)
    # init: listed destination rows zeroed, then the add
    e = y.copy()
    listed = np.zeros(n_cache, bool)
    listed[idx[:, 1] + off[1]] = True
    e.reshape(n_cache, W)[listed] = 0.0
    oracle.add_rows_from_double_index(e, x, idx, off, W, limit)
    ty = T(y, dev)
    plan.init(ty, T(x, dev))
    torch.cuda.synchronize()
    assert np.array_equal(bits(ty.cpu().numpy()), bits(e)), ("init", kind, W)
    plan.close()


@pytest.mark.parametrize("W,limit_frac", [(128, None), (64, 0.7), (130, None)])
def test_row_plan_repeated_destinations(dev, W, limit_frac):
    """An index listing destinations more than once (the reference's range
    check admits e.g. cache rows {0, 0, 2}, clientlib-viter.cpp:869-873):
    scatter plans add every occurrence in op order, as the CPU twin's loop
    does (row-op-util.hpp:121-139), so a dense run, a residual and repeat
    layers 1..3 together equal the oracle bit for bit; the fused init zeroes
    once, then adds in the same order; a gather plan with a repeated
    destination (id0) keeps the last assignment, as the CPU twin's loop does."""
    from geeps_amd import rowops
    rng = np.random.default_rng(W + 17)
    run = (4 << 20) // (W * 4) + 100  # one dense run of the plan's sweep size
    n_cache = run + 3000
    dense = np.stack([np.arange(run), np.arange(run)], 1)
    # 2000 more rows: destinations drawn from 700 rows (inside and outside the
    # run), so some appear 2-4 times; order interleaved with the run
    rep = rng.choice(np.concatenate([rng.choice(run, 300, replace=False), run + np.arange(400)]),
                     2000)
    extra = np.stack([run + np.arange(2000), rep], 1)
    # the run first in op order (its rows are the first occurrences of their
    # destinations, so it stays one dense run), then the rest shuffled
    idx = np.concatenate([dense, extra[rng.permutation(len(extra))]])
    n_op = len(idx)
    limit = None if limit_frac is None else int(n_op * W * limit_frac) + 5
    x = rng.standard_normal(n_op * W).astype(np.float32)
    y = rng.standard_normal(n_cache * W).astype(np.float32)
    plan = rowops.RowPlan(idx, n_op, (0, 0), W, limit)
    info = plan.info()
    counts = np.bincount(idx[:, 1], minlength=n_cache)
    assert info["repeat_rows"] == int((counts - 1).clip(0).sum())
    assert info["repeat_layers"] == int(counts.max()) - 1 >= 1
    assert info["dense_runs"] == (1 if limit is None else info["dense_runs"])
    e = y.copy()
    oracle.add_rows_from_double_index(e, x, idx, (0, 0), W, limit)
    ty = T(y, dev)
    plan.add(ty, T(x, dev))
    torch.cuda.synchronize()
    assert np.array_equal(bits(ty.cpu().numpy()), bits(e)), ("add", W)
    e = y.copy()
    e.reshape(n_cache, W)[counts > 0] = 0.0
    oracle.add_rows_from_double_index(e, x, idx, (0, 0), W, limit)
    ty = T(y, dev)
    plan.init(ty, T(x, dev))
    torch.cuda.synchronize()
    assert np.array_equal(bits(ty.cpu().numpy()), bits(e)), ("init", W)
    plan.close()
    # gather: y[id0] = x[id1], destination id0 repeated -> the last one wins
    g_idx = np.stack([rng.integers(0, 500, 1500), rng.integers(0, n_cache, 1500)], 1)
    g_lim = None if limit is None else 400 * W + 3
    src = rng.standard_normal(n_cache * W).astype(np.float32)
    out = rng.standard_normal(500 * W).astype(np.float32)
    e = out.copy()
    oracle.assign_rows_to_double_index(e, src, g_idx, (0, 0), W, g_lim)
    gplan = rowops.RowPlan(g_idx, len(g_idx), (0, 0), W, g_lim, kind="gather")
    assert gplan.info()["repeat_layers"] >= 1
    to = T(out, dev)
    gplan.gather(to, T(src, dev))
    torch.cuda.synchronize()
    assert np.array_equal(bits(to.cpu().numpy()), bits(e)), ("gather", W)
    gplan.close()


def test_row_plan_long_run_takes_sweep_forms(dev):
    """A 620,000-row dense run (303 MiB at 128 floats) moves through the sweep
    kernels: the add as 3 whole 96-MiB chunks (1 bucket) and the fused init as
    4 whole 64-MiB chunks of the zero-input form, each rest through the
    tile-major form; the run starts at x row 3 / y row 11, -0.0 deltas become
    +0.0 under init, and the last 100 rows (past num_vals_limit, one
    straddling it) plus 500 scattered rows take the residual path.  Bit for bit
    against the oracle (init: listed rows zeroed, then the add)."""
    import ctypes
    from geeps_amd import native, rowops
    rng = np.random.default_rng(620)
    W, run, scattered = 128, 620_000, 500
    n_op = run + scattered
    n_cache = n_op + 64
    dense = np.stack([3 + np.arange(run), 11 + np.arange(run)], 1)
    free = np.setdiff1d(np.arange(n_cache), dense[:, 1])
    extra = np.stack([np.setdiff1d(np.arange(n_op + 3), dense[:, 0])[:scattered],
                      rng.choice(free, scattered, replace=False)], 1)
    idx = np.concatenate([dense, extra])[rng.permutation(n_op)].astype(np.int64)
    limit = (3 + run - 100) * W + 37
    for nb, expect in ((1, 3),):
        launches, rt, sw = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_int(0)
        native.check(native.lib().gp_bucket_sum_sweep_plan((run - 100) * W, nb, ctypes.byref(launches),
                                                            ctypes.byref(rt), ctypes.byref(sw)))
        assert sw.value == expect and rt.value == 14
    x = rng.standard_normal((n_op + 3) * W).astype(np.float32)
    x[rng.choice(x.size, 5000, replace=False)] = np.float32(-0.0)
    y = rng.standard_normal(n_cache * W).astype(np.float32)
    plan = rowops.RowPlan(idx, n_op, (0, 0), W, limit)
    info = plan.info()
    assert info["dense_runs"] == 1 and info["dense_rows"] == run - 100
    e = y.copy()
    oracle.add_rows_from_double_index(e, x, idx, (0, 0), W, limit)
    ty = T(y, dev)
    plan.add(ty, T(x, dev))
    torch.cuda.synchronize()
    assert np.array_equal(bits(ty.cpu().numpy()), bits(e)), "add"
    e = y.copy()
    listed = np.zeros(n_cache, bool)
    listed[idx[:, 1]] = True
    e.reshape(n_cache, W)[listed] = 0.0
    oracle.add_rows_from_double_index(e, x, idx, (0, 0), W, limit)
    ty = T(y, dev)
    plan.init(ty, T(x, dev))
    torch.cuda.synchronize()
    assert np.array_equal(bits(ty.cpu().numpy()), bits(e)), "init"
    plan.close()


@pytest.mark.parametrize("kind", ["identity", "permuted", "mixed"])
@pytest.mark.parametrize("W,limit_frac,off,nseg", [(128, None, (0, 0), 0), (64, None, (5, 3), 0),
                                                    (128, 0.83, (0, 0), 0), (1024, None, (0, 2), 0),
                                                    (130, None, (0, 0), 0), (4, 0.5, (1, 1), 0),
                                                    (128, None, (0, 0), 3), (128, 0.9, (2, 1), 7),
                                                    (64, None, (0, 0), 64)])
def test_gather_plan_matches_oracle(dev, kind, W, limit_frac, off, nseg):
    """gp_gather_rows_planned / gp_gather_rows_segmented_planned (the Read
    side's plan: dense runs copied by the phase-separated kernels, the rest by
    the gather row kernels in destination order) equal the oracle's
    assign_rows_to_double_index bit for bit, with offsets, num_vals_limit on
    the destination, and segment boundaries cutting the dense runs; rows not
    listed are untouched (the scatter plans' indexes: the mixed case has 3
    dense runs of >= 4 MiB, short runs and scattered rows)."""
    from geeps_amd import rowops
    rng = np.random.default_rng(W * 5 + len(kind) + nseg + int((limit_frac or 0) * 10))
    n_cache = 5 * ((4 << 20) // (W * 4)) + 8000
    # id0: op-buffer rows (the destinations, distinct), id1: cache rows
    idx, n_op = _plan_index(rng, kind, n_cache - off[1], W)
    n_y = int(idx[:, 0].max()) + 1 + off[0] + 3
    limit = None if limit_frac is None else int(n_y * W * limit_frac) + 3
    x = rng.standard_normal(n_cache * W).astype(np.float32)
    x[rng.choice(x.size, 300, replace=False)] = np.float32(-0.0)
    y = rng.standard_normal(n_y * W).astype(np.float32)
    e = y.copy()
    oracle.assign_rows_to_double_index(e, x, idx, off, W, limit)
    plan = rowops.RowPlan(idx, n_op, off, W, limit, kind="gather")
    info = plan.info()
    if kind == "identity" and limit is None:
        assert info == {"rows": n_op, "dense_runs": 1, "dense_rows": n_op, "residual_rows": 0,
                        "repeat_layers": 0, "repeat_rows": 0}
    if kind == "mixed" and limit is None:
        assert info["dense_runs"] == 3 and info["residual_rows"] > 0
    ty = T(y, dev)
    if nseg == 0:
        plan.gather(ty, T(x, dev))
    else:
        bounds = _split(rng, n_cache, nseg)
        segs = [(bounds[i], T(x[bounds[i] * W:bounds[i + 1] * W], dev)) for i in range(nseg)]
        plan.gather_segmented(ty, segs)
    torch.cuda.synchronize()
    assert np.array_equal(bits(ty.cpu().numpy()), bits(e)), (kind, W, nseg)
    with pytest.raises(ValueError):
        plan.add(ty, T(x, dev))
    plan.close()


def test_gather_plan_long_run_takes_sweep(dev):
    """A 420,000-row identity-like gather (205 MiB at 128 floats: 3 whole
    64-MiB copy sweeps, then the tile-major rest) from a cache split in 2
    segments at a row inside the run: bit for bit, -0.0 and NaN payloads
    copied unchanged."""
    import ctypes
    from geeps_amd import native, rowops
    rng = np.random.default_rng(42)
    W, n = 128, 420_000
    idx = np.stack([np.arange(n), 9 + np.arange(n)], 1).astype(np.int64)
    x = rng.standard_normal((n + 20) * W).astype(np.float32)
    x[:5000] = np.float32(-0.0)
    x.view(np.uint32)[5000:5010] = 0x7FC00123  # NaN with a payload
    y = np.zeros(n * W, np.float32)
    plan = rowops.RowPlan(idx, row_size=W, kind="gather")
    a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    native.check(native.lib().gp_row_plan_launches(plan._h, 0, ctypes.byref(a), ctypes.byref(b),
                                                   ctypes.byref(c)))
    assert a.value == 3 and b.value == 1
    cut = 9 + 250_000
    segs = [(0, T(x[:cut * W], dev)), (cut, T(x[cut * W:], dev))]
    ty = T(y, dev)
    plan.gather_segmented(ty, segs)
    torch.cuda.synchronize()
    assert np.array_equal(bits(ty.cpu().numpy()), bits(x[9 * W:(9 + n) * W]))
    ty.zero_()
    plan.gather(ty, T(x, dev))
    torch.cuda.synchronize()
    assert np.array_equal(bits(ty.cpu().numpy()), bits(x[9 * W:(9 + n) * W]))
    plan.close()


def _fuzz_index(rng, n_cache, W):
    """An op index built from random pieces: dense runs (some past the 4-MiB
    plan threshold), short runs, single rows, in shuffled op order; id0 are
    the op rows (distinct), id1 distinct cache rows."""
    big = max(1, (4 << 20) // (W * 4))
    free = rng.permutation(n_cache)
    taken = np.zeros(n_cache, bool)
    parts, j0 = [], 0
    for _ in range(int(rng.integers(1, 6))):
        L = int(rng.choice([1, 2, 7, big - 1, big, big + 13, 2 * big]))
        start = int(rng.integers(0, max(1, n_cache - L)))
        seg = np.arange(start, min(n_cache, start + L))
        seg = seg[~taken[seg]]
        if seg.size == 0:
            continue
        # keep only the longest stretch of consecutive untaken rows
        cuts = np.flatnonzero(np.diff(seg) != 1) + 1
        seg = max(np.split(seg, cuts), key=len)
        taken[seg] = True
        parts.append(np.stack([j0 + np.arange(seg.size), seg], 1))
        j0 += seg.size
    rest = free[~taken[free]][:int(rng.integers(0, 2000))]
    if rest.size:
        parts.append(np.stack([j0 + np.arange(rest.size), rest], 1))
        j0 += rest.size
    idx = np.concatenate(parts).astype(np.int64)
    return idx[rng.permutation(idx.shape[0])], idx.shape[0]


# GEEPS_FUZZ_CASES=<n> widens the fuzzed parity tests below (a one-off
# campaign, scripts/gpu_runs/r03/fuzz.sh); the default keeps the suite short.
_FUZZ_CASES = int(os.environ.get("GEEPS_FUZZ_CASES", "24"))


@pytest.mark.parametrize("case", range(_FUZZ_CASES))
def test_row_plans_fuzz(dev, case):
    """Random op indexes (dense runs around the plan threshold, short runs,
    scattered rows), row sizes, offsets and num_vals_limit: the scatter plan's
    add and init and the gather plan's flat and segmented gather (segments
    16-B aligned or not) all equal the oracle bit for bit."""
    from geeps_amd import rowops
    rng = np.random.default_rng(9000 + case)
    W = int(rng.choice([4, 8, 64, 128, 132, 256]))
    n_cache = 3 * max(1, (4 << 20) // (W * 4)) + int(rng.integers(100, 5000))
    off = (int(rng.integers(0, 4)), int(rng.integers(0, 4)))
    idx, n_op = _fuzz_index(rng, n_cache - off[1], W)
    n_x = n_op + off[0]
    limit = None if rng.random() < 0.5 else int(rng.integers(1, n_x * W + 1))
    x = rng.standard_normal(n_x * W).astype(np.float32)
    x[rng.choice(x.size, min(x.size, 200), replace=False)] = np.float32(-0.0)
    y = rng.standard_normal(n_cache * W).astype(np.float32)
    tx = T(x, dev)
    # scatter plan: add, init
    plan = rowops.RowPlan(idx, n_op, off, W, limit)
    e = y.copy()
    oracle.add_rows_from_double_index(e, x, idx, off, W, limit)
    ty = T(y, dev)
    plan.add(ty, tx)
    torch.cuda.synchronize()
    assert np.array_equal(bits(ty.cpu().numpy()), bits(e)), ("add", case, W, off, limit)
    e = y.copy()
    listed = np.zeros(n_cache, bool)
    listed[idx[:, 1] + off[1]] = True
    e.reshape(n_cache, W)[listed] = 0.0
    oracle.add_rows_from_double_index(e, x, idx, off, W, limit)
    ty = T(y, dev)
    plan.init(ty, tx)
    torch.cuda.synchronize()
    assert np.array_equal(bits(ty.cpu().numpy()), bits(e)), ("init", case, W, off, limit)
    plan.close()
    # gather plan: y_op[id0] = cache[id1], the limit on the op side
    gplan = rowops.RowPlan(idx, n_op, off, W, limit, kind="gather")
    cache = y
    dst = rng.standard_normal(n_x * W).astype(np.float32)
    e = dst.copy()
    oracle.assign_rows_to_double_index(e, cache, idx, off, W, limit)
    td = T(dst, dev)
    gplan.gather(td, T(cache, dev))
    torch.cuda.synchronize()
    assert np.array_equal(bits(td.cpu().numpy()), bits(e)), ("gather", case, W, off, limit)
    nseg = int(rng.integers(1, 9))
    bounds = _split(rng, n_cache, nseg)
    pad = int(rng.integers(0, 2))  # 1: every segment a view one float into its buffer (unaligned)

    def seg(i):
        a, b = bounds[i] * W, bounds[i + 1] * W
        big = torch.empty(b - a + pad, dtype=torch.float32, device=dev)
        big[pad:].copy_(T(cache[a:b], dev))
        return big[pad:]

    segs = [(bounds[i], seg(i)) for i in range(nseg)]
    td = T(dst, dev)
    gplan.gather_segmented(td, segs)
    torch.cuda.synchronize()
    assert np.array_equal(bits(td.cpu().numpy()), bits(e)), ("gather_seg", case, W, off, limit, nseg)
    gplan.close()


def test_row_plan_unaligned_and_side_stream(dev):
    """Bases 4 B off 16-B alignment (a dense run takes the scalar sum form, the
    residual the scalar row kernel) on a side stream: still bit-exact."""
    from geeps_amd import rowops
    rng = np.random.default_rng(9)
    W, n = 128, 20000
    idx = np.stack([np.arange(n), np.arange(n)], 1).astype(np.int64)
    idx[12000:] = idx[12000:][rng.permutation(n - 12000)]
    idx[12000:, 0] = np.arange(12000, n)
    x = rng.standard_normal(n * W + 1).astype(np.float32)
    y = rng.standard_normal(n * W + 1).astype(np.float32)
    e = y[1:].copy()
    oracle.add_rows_from_double_index(e, x[1:].copy(), idx, (0, 0), W)
    plan = rowops.RowPlan(idx, row_size=W)
    assert plan.info()["dense_runs"] == 1 and plan.info()["residual_rows"] == n - 12000
    ty, tx = T(y, dev), T(x, dev)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        plan.add(ty[1:], tx[1:])
    s.synchronize()
    assert np.array_equal(bits(ty.cpu().numpy()[1:]), bits(e))
    assert ty[0].item() == y[0]


def test_row_plan_rejects_small_buffers(dev):
    from geeps_amd import rowops
    idx = np.stack([np.arange(10), np.arange(10) + 5], 1)
    plan = rowops.RowPlan(idx, row_size=128)
    with pytest.raises(ValueError):
        plan.add(torch.zeros(14 * 128, device=dev), torch.zeros(10 * 128, device=dev))
    with pytest.raises(ValueError):
        plan.add(torch.zeros(15 * 128, device=dev), torch.zeros(9 * 128, device=dev))


@pytest.mark.parametrize("N,out_of_place", [(3, False), (3, True), (7, False), (7, True)])
def test_bucket_sum_sweep_then_small_leftover(dev, N, out_of_place):
    """3 whole 64-MiB sweep chunks, then a 1-MiB leftover (below the phased
    form's 4 MiB: the mixed dwordx4 form at offset `done`) and a 3-float scalar
    tail, at 3 and 7 buckets, in place and out of place."""
    import ctypes
    from geeps_amd import native, rowops
    n = (48 << 20) + (1 << 18) + 3
    launches, rt, sw = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_int(0)
    native.check(native.lib().gp_bucket_sum_sweep_plan(n, N, ctypes.byref(launches),
                                                        ctypes.byref(rt), ctypes.byref(sw)))
    assert (sw.value, launches.value) == (3, 3)
    ups = [oracle.synthetic_delta(700 + c, n) for c in range(N)]
    m0 = np.random.default_rng(N + 40).standard_normal(n).astype(np.float32)
    e = m0.copy()
    oracle.apply_updates(e, ups)
    m = T(m0, dev)
    tb = [T(u, dev) for u in ups]
    if out_of_place:
        out = torch.full((n,), float("nan"), dtype=torch.float32, device=dev)
        rowops.bucket_sum_into(out, m, tb)
        torch.cuda.synchronize()
        assert np.array_equal(bits(m.cpu().numpy()), bits(m0))
    else:
        rowops.bucket_sum_apply(m, tb)
        out = m
    torch.cuda.synchronize()
    assert np.array_equal(bits(out.cpu().numpy()), bits(e))


def test_c_abi_consumer_on_gpu(dev):
    """tests/apps/c_abi_check.c — a plain C99 program calling the C-ABI (built by
    __graft_entry__.build() with gcc): the 8-way bucket sum, the scatter-add
    (op order and row plan), the fused init and the gather (flat and planned),
    each bit-exact against the oracle, from C with no torch or HIP type."""
    import os
    import subprocess
    from conftest import REPO
    exe = os.path.join(REPO, "build", "tests", "c_abi_check")
    assert os.path.exists(exe), "run __graft_entry__.build() first"
    torch.cuda.synchronize()
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "c_abi_check ok" in r.stdout, r.stdout + r.stderr
    for what in ("gp_bucket_sum_apply 8 buckets", "gp_scatter_add_rows", "gp_scatter_add_rows_planned",
                 "gp_scatter_init_rows_planned", "gp_gather_rows", "gp_gather_rows_planned"):
        assert f"{what}: " in r.stdout and "bit-exact" in r.stdout


# Sizes around the plan's boundaries on 256 CUs (floats): 3 whole 96-MiB chunks
# (the big sweep's threshold), 3 whole 64-MiB chunks, whole multiples of both,
# each +- one 16-KiB tile per block, one dwordx4 and single floats.
_MiB = 1 << 18  # floats per MiB
_FUZZ_SIZES = [3 * 96 * _MiB, 3 * 96 * _MiB - 4, 3 * 96 * _MiB + 4 * 1024 * 256 + 5,
               3 * 64 * _MiB, 3 * 64 * _MiB - 1, 2 * 96 * _MiB + 64 * _MiB + 3,
               5 * 96 * _MiB + 2 * 64 * _MiB + 7, 4 * 96 * _MiB + 17 * _MiB + 1]


@pytest.mark.parametrize("case", range(16))
def test_bucket_sum_plan_boundaries_fuzz(dev, case):
    """Random bucket counts (1-8, and 9-11 for chained passes) and in-place /
    out-of-place sums at sizes around the launch plan's boundaries: every
    element bit for bit against a plain torch fp32 reference adding the buckets
    in client order, and the input left untouched out of place."""
    from geeps_amd import rowops
    rng = np.random.default_rng(9000 + case)
    n = int(_FUZZ_SIZES[case % len(_FUZZ_SIZES)])
    N = int(rng.integers(1, 12)) if case % 4 == 3 else int(rng.integers(1, 9))
    out_of_place = bool(case % 2)
    g = torch.Generator(device=dev)
    g.manual_seed(9000 + case)
    buckets = [torch.rand(n, generator=g, device=dev) - 0.5 for _ in range(N)]
    master = torch.rand(n, generator=g, device=dev) - 0.5
    expect = master.clone()
    for b in buckets:
        expect += b
    if out_of_place:
        m0 = master.clone()
        out = torch.full((n,), float("nan"), dtype=torch.float32, device=dev)
        rowops.bucket_sum_into(out, master, buckets)
        torch.cuda.synchronize()
        assert torch.equal(master.view(torch.int32), m0.view(torch.int32))
    else:
        rowops.bucket_sum_apply(master, buckets)
        out = master
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int32), expect.view(torch.int32)), (n, N, out_of_place)


@pytest.mark.parametrize("case", range(max(6, _FUZZ_CASES // 4)))
def test_unplanned_calls_fuzz(analyzed, dev, case):
    """The reference binding's unplanned calls through the device plan and
    its plan cache, on fuzzed indexes (dense runs around the sweep threshold,
    short runs, scattered rows, in shuffled op order), row sizes, offsets and
    num_vals_limit: three scatter-adds (the first builds the plan: an inverse
    map at up to 128 floats a row, else op order and, on the second call, the
    sorted residual; later ones run it behind the device check), then two more
    after two destinations of the index were swapped in place (the steady
    state's gated op-order form, then the re-plan), three inits, and three
    gathers plus two after a swap of two sources (the ranges plan's steady
    state and its select launch), each bit for bit against the oracle."""
    from geeps_amd import rowops
    rng = np.random.default_rng(7000 + case)
    W = int(rng.choice([4, 64, 128, 132, 256]))
    n_cache = 3 * max(1, (4 << 20) // (W * 4)) + int(rng.integers(100, 5000))
    off = (int(rng.integers(0, 4)), int(rng.integers(0, 4)))
    idx, n_op = _fuzz_index(rng, n_cache - off[1], W)
    n_x = n_op + off[0]
    limit = None if rng.random() < 0.5 else int(rng.integers(1, n_x * W + 1))
    x = rng.standard_normal(n_x * W).astype(np.float32)
    x[rng.choice(x.size, min(x.size, 200), replace=False)] = np.float32(-0.0)
    y = rng.standard_normal(n_cache * W).astype(np.float32)
    tx, ti = T(x, dev), torch.from_numpy(idx).to(dev)
    e = y.copy()
    oracle.add_rows_from_double_index(e, x, idx, off, W, limit)
    for call in range(3):
        ty = T(y, dev)
        rowops.add_rows_from_double_index_gpu(ty, tx, ti, n_op, off, W, limit)
        torch.cuda.synchronize()
        assert np.array_equal(bits(ty.cpu().numpy()), bits(e)), ("add", case, call, W, off, limit)
    # the same tensor, two destinations swapped (still distinct)
    idx2 = idx.copy()
    a, b = rng.choice(n_op, 2, replace=False)
    idx2[[a, b], 1] = idx2[[b, a], 1]
    ti.copy_(torch.from_numpy(idx2))
    e = y.copy()
    oracle.add_rows_from_double_index(e, x, idx2, off, W, limit)
    for call in range(2):
        ty = T(y, dev)
        rowops.add_rows_from_double_index_gpu(ty, tx, ti, n_op, off, W, limit)
        torch.cuda.synchronize()
        assert np.array_equal(bits(ty.cpu().numpy()), bits(e)), ("add changed", case, call, W, off, limit)
    ti.copy_(torch.from_numpy(idx))
    e = y.copy()
    e.reshape(n_cache, W)[idx[:, 1] + off[1]] = 0.0
    oracle.add_rows_from_double_index(e, x, idx, off, W, limit)
    for call in range(3):
        ty = T(y, dev)
        rowops.init_rows_from_double_index_gpu(ty, tx, ti, n_op, off, W, limit)
        torch.cuda.synchronize()
        assert np.array_equal(bits(ty.cpu().numpy()), bits(e)), ("init", case, call, W, off, limit)
    # gathers: the first plans (runs and residual ranges), later ones run it
    # behind the device check; then two sources swapped in place
    dst = rng.standard_normal(n_x * W).astype(np.float32)
    ty = T(y, dev)
    for changed in (False, True):
        if changed:
            gidx = idx.copy()
            gidx[[a, b], 1] = gidx[[b, a], 1]
            ti.copy_(torch.from_numpy(gidx))
        else:
            gidx = idx
        e = dst.copy()
        oracle.assign_rows_to_double_index(e, y, gidx, off, W, limit)
        for call in range(3 if not changed else 2):
            td = T(dst, dev)
            rowops.assign_rows_to_double_index_gpu(td, ty, ti, n_op, off, W, limit)
            torch.cuda.synchronize()
            assert np.array_equal(bits(td.cpu().numpy()), bits(e)), ("gather", changed, call, case, W, off, limit)

