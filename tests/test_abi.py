"""The C-ABI library loads and exports every symbol include/gp_reduce.h declares
(no compute calls: runs without a GPU)."""
import ctypes
import os
import subprocess

from conftest import REPO

from geeps_amd import native


def test_header_declares_expected_entry_points():
    syms = native.declared_symbols()
    for s in ("gp_scatter_add_rows", "gp_gather_rows", "gp_scatter_rows",
              "gp_bucket_sum_apply", "gp_bucket_sum_into", "gp_bucket_sum_plan", "gp_bucket_sum_sweep_plan", "gp_add", "gp_zero",
              "gp_last_error"):
        assert s in syms
    # every declared symbol has a ctypes signature and vice versa
    assert set(syms) == set(native._SIGNATURES)


def test_library_exports_every_declared_symbol():
    assert os.path.exists(native.LIB_PATH), "run __graft_entry__.build() first"
    out = subprocess.run(["nm", "-D", "--defined-only", native.LIB_PATH], check=True,
                         capture_output=True, text=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [s for s in native.declared_symbols() if s not in exported]
    assert not missing, missing


def test_library_loads_and_reports_abi():
    L = native.lib()
    assert L.gp_abi_version() == native.ABI_VERSION == 16
    assert isinstance(L.gp_last_error(), bytes)


def test_library_is_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", native.LIB_PATH],
                         capture_output=True, text=True).stdout
    assert ".hip_fatbin" in out
    blob = open(native.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_invalid_arguments_rejected_without_device():
    # argument validation happens before any HIP call
    L = native.lib()
    rc = L.gp_bucket_sum_apply(None, None, 2, 16, None)
    assert rc == 1 and b"null" in L.gp_last_error()
    rc = L.gp_scatter_add_rows(ctypes.c_void_p(16), ctypes.c_void_p(16), ctypes.c_void_p(16), 4,
                               native.DoubleIndex(0, 0), 0, 100, None)
    assert rc == 1 and b"row_size" in L.gp_last_error()
    # zero-size calls are no-ops that never touch the device
    assert L.gp_bucket_sum_apply(None, None, 0, 16, None) == 0
    # out-of-place form: nulls and overlapping out / in are rejected before any launch
    assert L.gp_bucket_sum_into(None, ctypes.c_void_p(4096), None, 1, 16, None) == 1
    assert L.gp_bucket_sum_into(ctypes.c_void_p(4096 + 16), ctypes.c_void_p(4096), None, 0, 16,
                                None) == 1
    assert b"overlap" in L.gp_last_error()
    assert L.gp_bucket_sum_into(None, None, None, 1, 0, None) == 0
    assert L.gp_scatter_add_rows(None, None, None, 0, native.DoubleIndex(0, 0), 128, 0, None) == 0


def test_segment_tables_rejected_without_device():
    L = native.lib()
    p = ctypes.c_void_p(4096)
    idx = ctypes.c_void_p(4096)
    t = native.RowSegments()

    def gather():
        return L.gp_gather_rows_segmented(p, t, idx, 4, native.DoubleIndex(0, 0), 128, 1 << 40, None)

    def add():
        return L.gp_scatter_add_rows_segmented(t, p, idx, 4, native.DoubleIndex(0, 0), 128, 1 << 40,
                                               None)

    t.count = 0
    assert gather() == native.GP_ERR_INVALID and b"count" in L.gp_last_error()
    t.count = native.GP_MAX_SEGMENTS + 1
    assert add() == native.GP_ERR_INVALID and b"count" in L.gp_last_error()
    t.count = 2
    t.first_row[0], t.first_row[1] = 1, 5
    t.base[0] = t.base[1] = 4096
    assert gather() == native.GP_ERR_INVALID and b"first_row[0]" in L.gp_last_error()
    t.first_row[0], t.first_row[1] = 0, 0
    assert add() == native.GP_ERR_INVALID and b"ascending" in L.gp_last_error()
    t.first_row[1] = 5
    t.base[1] = None
    assert gather() == native.GP_ERR_INVALID and b"null" in L.gp_last_error()
    assert L.gp_gather_rows_segmented(p, None, idx, 4, native.DoubleIndex(0, 0), 128, 1, None) \
        == native.GP_ERR_INVALID
    # zero rows: a no-op before any check
    assert L.gp_gather_rows_segmented(None, None, None, 0, native.DoubleIndex(0, 0), 128, 1,
                                      None) == native.GP_OK


def test_product_does_not_import_oracle():
    """No product source imports, links or calls the CPU oracle."""
    import re
    pat = re.compile(r"^\s*(from\s+oracle|import\s+oracle)|liboracle|oracle_\w+\s*\(|oracle\.\w+\(",
                     re.M)
    for root, _, files in os.walk(os.path.join(REPO, "geeps_amd")):
        for f in files:
            if f.endswith((".py", ".cpp", ".hpp", ".hip", ".h")) or f == "Makefile":
                text = open(os.path.join(root, f)).read()
                assert not pat.search(text), os.path.join(root, f)
    for lib in ("libgp_reduce.so", "libgeeps.so"):
        p = os.path.join(REPO, "geeps_amd", "lib", lib)
        if os.path.exists(p):
            out = subprocess.run(["nm", "-D", p], capture_output=True, text=True).stdout
            assert "oracle_" not in out
            deps = subprocess.run(["readelf", "-d", p], capture_output=True, text=True).stdout
            assert "liboracle" not in deps


def test_bucket_sum_plan_without_device():
    """gp_bucket_sum_plan launches nothing.  Without a device the library
    assumes MI355X's 256 CUs, as on the GPU box; chunk sizes there: 96 MiB
    for the sweep form (7 register tiles of 32 KiB at 2-8 buckets, 14 of 16
    KiB at 1, beside 160 KiB of LDS per block), then 64 MiB at 3-8 buckets (6
    register tiles of 16 KiB), on shards of at least 3 such chunks;
    tile-major 56 / 88 / 120 MiB
    with 4 / 12 / 20 register tiles for the rest; balanced chunks from 4 MiB
    (one 16-KiB tile per block) up."""
    L = native.lib()
    launches, rt = ctypes.c_int(-5), ctypes.c_int(-5)

    def plan(n, nb):
        assert L.gp_bucket_sum_plan(n, nb, ctypes.byref(launches), ctypes.byref(rt)) == 0
        return launches.value, rt.value

    sweeps = ctypes.c_int(-5)

    def sweep_plan(n, nb):
        assert L.gp_bucket_sum_sweep_plan(n, nb, ctypes.byref(launches), ctypes.byref(rt),
                                          ctypes.byref(sweeps)) == 0
        return launches.value, rt.value, sweeps.value

    # the 4 GiB headline shard: 42 sweep chunks of 96 MiB, then one of 64 MiB
    assert sweep_plan(1 << 30, 8) == (43, 7, 43)
    assert plan(1 << 30, 8) == (43, 7)
    # 1-2 buckets: the rest after the 96-MiB chunks goes to the tile-major form
    assert sweep_plan(1 << 30, 2) == (43, 7, 42)
    assert sweep_plan(1 << 30, 1) == (43, 14, 42)
    assert sweep_plan(1 << 30, 4) == (43, 7, 43)
    assert sweep_plan(288 << 18, 2) == (3, 7, 3)
    # the 8-GPU shard (512 MiB): 4 x 96 + 2 x 64 MiB (not 5 x 96 + a 32-MiB tile-major rest)
    assert sweep_plan(1 << 27, 8) == (6, 7, 6)
    assert sweep_plan(1 << 29, 8) == (22, 7, 22)  # the 2-GPU shard: 20 x 96 + 2 x 64 MiB
    assert sweep_plan(1 << 28, 3) == (11, 7, 11)  # the 4-GPU shard (1 GiB): 10 x 96 + 64 MiB
    # 200 MiB: under 3 big chunks, so 3 64-MiB sweep chunks, then the 8-MiB
    # rest in 1 balanced tile-major chunk
    assert sweep_plan(200 << 18, 8) == (4, 6, 3)
    assert sweep_plan(120 << 18, 8) == (3, 4, 0)  # under 3 sweep chunks: tile-major only
    # below 3 register-form chunks: <= 3 balanced chunks of the same form, one per launch
    assert plan(3 * 10 * 1024 * 1024, 8) == (3, 4)   # 120 MiB: 7,680 tiles / 3,584 per chunk
    assert plan(30 << 18, 5) == (1, 4)
    assert plan(30 << 18, 4) == (1, 12)
    assert plan(200 << 18, 1) == (2, 20)
    assert plan(1 << 20, 8) == (1, 4)        # 4 MiB: one tile per block
    assert plan((1 << 20) - 4, 8) == (0, -1)  # below: the mixed form
    assert plan(0, 1) == (0, -1)
    assert L.gp_bucket_sum_plan(16, 9, ctypes.byref(launches), ctypes.byref(rt)) == 1
    assert L.gp_bucket_sum_plan(16, 0, ctypes.byref(launches), ctypes.byref(rt)) == 1
    assert L.gp_bucket_sum_plan(16, 1, None, None) == 1
    # every launch by form
    sp = native.SumPlan()
    assert L.gp_bucket_sum_launch_plan(1 << 30, 8, ctypes.byref(sp)) == 0
    assert (sp.sweep_launches, sp.sweep_reg_tiles, sp.small_sweep_launches, sp.phased_launches,
            sp.phased_reg_tiles, sp.other_launches) == (42, 7, 1, 0, -1, 0)
    # 2-8 buckets: 32-KiB tiles, bursts of 1; the 64-MiB chunks: 16-KiB tiles, bursts of 4
    assert (sp.sweep_burst_tiles, sp.sweep_tile_kib, sp.small_sweep_burst_tiles) == (1, 32, 4)
    assert L.gp_bucket_sum_launch_plan(1 << 30, 2, ctypes.byref(sp)) == 0
    assert (sp.sweep_launches, sp.sweep_reg_tiles, sp.sweep_burst_tiles, sp.sweep_tile_kib,
            sp.small_sweep_launches, sp.small_sweep_burst_tiles) == (42, 7, 1, 32, 0, -1)  # no 64-MiB chunks
    assert L.gp_bucket_sum_launch_plan(1 << 30, 1, ctypes.byref(sp)) == 0
    assert (sp.sweep_launches, sp.sweep_reg_tiles, sp.sweep_burst_tiles, sp.sweep_tile_kib,
            sp.small_sweep_launches) == (42, 14, 8, 16, 0)  # 1 bucket: 16-KiB tiles, bursts of 8
    n = (1 << 27) + 4 + 3  # 512 MiB + one dwordx4 + 3 floats
    assert L.gp_bucket_sum_launch_plan(n, 5, ctypes.byref(sp)) == 0
    assert (sp.sweep_launches, sp.small_sweep_launches, sp.phased_launches, sp.phased_reg_tiles,
            sp.other_launches) == (4, 2, 0, -1, 2)
    n = (1 << 27) + (16 << 18)  # 528 MiB: 4 x 96 + 2 x 64 MiB, 16 MiB tile-major (not 48)
    assert L.gp_bucket_sum_launch_plan(n, 5, ctypes.byref(sp)) == 0
    assert (sp.sweep_launches, sp.small_sweep_launches, sp.phased_launches, sp.phased_reg_tiles,
            sp.other_launches) == (4, 2, 1, 4, 0)
    n = (1 << 27) + (64 << 18)  # 576 MiB = 6 x 96 MiB exactly
    assert L.gp_bucket_sum_launch_plan(n, 8, ctypes.byref(sp)) == 0
    assert (sp.sweep_launches, sp.small_sweep_launches, sp.phased_launches) == (6, 0, 0)
    assert L.gp_bucket_sum_launch_plan(n, 9, ctypes.byref(sp)) == 1
    assert L.gp_bucket_sum_launch_plan(n, 2, None) == 1


def _plan(idx, offset=(0, 0), row_size=128, limit=None):
    import numpy as np
    L = native.lib()
    h = ctypes.c_void_p()
    a = np.ascontiguousarray(idx, dtype=np.int64)
    rc = L.gp_row_plan_create(ctypes.byref(h), a.ctypes.data, a.shape[0], native.DoubleIndex(*offset),
                              row_size, (1 << 64) - 1 if limit is None else limit)
    return rc, h


def _info(h):
    a, b, c = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
    assert native.lib().gp_row_plan_info(h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)) == 0
    return a.value, b.value, c.value


def test_row_plan_launches_without_device():
    """gp_row_plan_launches reports what a planned add / init issues (no
    device: an index that is one dense run allocates nothing).  The 4 GiB
    identity plan (1M rows of 1024 floats): the add as 42 sweep chunks of 96
    MiB + the 64-MiB rest tile-major, the init as 64 zero-input sweep chunks of
    64 MiB."""
    import numpy as np
    n = 1 << 20
    rc, h = _plan(np.stack([np.arange(n), np.arange(n)], 1), row_size=1024)
    assert rc == 0
    a, b, c = ctypes.c_int(-1), ctypes.c_int(-1), ctypes.c_int(-1)

    def launches(plan, init):
        assert native.lib().gp_row_plan_launches(plan, init, ctypes.byref(a), ctypes.byref(b),
                                                 ctypes.byref(c)) == 0
        return a.value, b.value, c.value

    assert launches(h, 0) == (42, 1, 0)
    assert launches(h, 1) == (64, 0, 0)
    assert native.lib().gp_row_plan_destroy(h) == 0
    # a 4.9-MiB run: one balanced tile-major chunk (312 whole tiles on 256
    # CUs), then the half tile left in one mixed-form launch
    rc, h = _plan(np.stack([np.arange(10000), 7 + np.arange(10000)], 1), row_size=128)
    assert rc == 0 and _info(h) == (10000, 1, 10000)
    assert launches(h, 0) == (0, 1, 1) and launches(h, 1) == (0, 1, 1)
    assert native.lib().gp_row_plan_destroy(h) == 0
    assert native.lib().gp_row_plan_launches(None, 0, ctypes.byref(a), ctypes.byref(b),
                                             ctypes.byref(c)) == 1


def test_gather_plan_without_device():
    """Gather plans (gp_gather_plan_create): destinations are id0; an identity index is one dense run, copied by the no-bucket
    sweep in 64-MiB chunks (a 4 GiB table: 64 launches); plans of one kind
    are refused by the other kind's calls before anything launches."""
    import numpy as np
    L = native.lib()
    h = ctypes.c_void_p()
    n = 1 << 20
    a = np.ascontiguousarray(np.stack([np.arange(n), 5 + np.arange(n)], 1), dtype=np.int64)
    assert L.gp_gather_plan_create(ctypes.byref(h), a.ctypes.data, n, native.DoubleIndex(0, 0), 1024,
                                   (1 << 64) - 1) == 0
    assert _info(h) == (n, 1, n)
    x, y, z = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    assert L.gp_row_plan_launches(h, 0, ctypes.byref(x), ctypes.byref(y), ctypes.byref(z)) == 0
    assert (x.value, y.value, z.value) == (64, 0, 0)
    # a gather plan is not a scatter plan, and the other way round
    fake = ctypes.c_void_p(16)
    assert L.gp_scatter_add_rows_planned(fake, fake, h, None) == 1
    assert b"gather row plan" in L.gp_last_error()
    assert L.gp_row_plan_destroy(h) == 0
    rc, hs = _plan(a, row_size=1024)
    assert rc == 0
    assert L.gp_gather_rows_planned(fake, fake, hs, None) == 1
    assert b"scatter row plan" in L.gp_last_error()
    assert L.gp_row_plan_destroy(hs) == 0
    # a repeated destination row (id0) goes to a repeat layer (device memory:
    # without a device the allocation fails, the index is not refused)
    dup = np.ascontiguousarray([[0, 1], [1, 2], [1, 3]], dtype=np.int64)
    rc = L.gp_gather_plan_create(ctypes.byref(h), dup.ctypes.data, 3, native.DoubleIndex(0, 0), 128,
                                 (1 << 64) - 1)
    assert b"repeat" not in L.gp_last_error()
    if rc == 0:
        assert L.gp_row_plan_destroy(h) == 0
    else:
        assert rc == native.GP_ERR_HIP


def test_row_plan_classifies_dense_runs_without_device():
    """Plans whose rows all fall in dense runs need no device memory, so the
    host-side classifier runs here: runs of >= 4 MiB where id0 and id1 both
    step by one, found after sorting by id1 (any op row order), offsets
    applied; empty plans too."""
    import numpy as np
    L = native.lib()
    R = 8192  # one 4-MiB run at 128 floats
    rc, h = _plan(np.stack([np.arange(R), np.arange(R)], 1))
    assert rc == 0 and _info(h) == (R, 1, R)
    L.gp_row_plan_destroy(h)
    # two runs listed in reverse op order, the second's destinations below the first's
    two = np.concatenate([np.stack([np.arange(R), 5 * R + np.arange(R)], 1),
                          np.stack([R + np.arange(R), np.arange(R)], 1)])[::-1]
    rc, h = _plan(two, offset=(3, 7))
    assert rc == 0 and _info(h) == (2 * R, 2, 2 * R)
    L.gp_row_plan_destroy(h)
    # 64-float rows: a run needs 16384 rows
    rc, h = _plan(np.stack([np.arange(2 * R), np.arange(2 * R)], 1), row_size=64)
    assert rc == 0 and _info(h) == (2 * R, 1, 2 * R)
    L.gp_row_plan_destroy(h)
    rc, h = _plan(np.zeros((0, 2)))
    assert rc == 0 and _info(h) == (0, 0, 0)
    assert L.gp_row_plan_destroy(h) == 0
    assert L.gp_row_plan_destroy(None) == 0
    assert L.gp_row_plan_info(None, None, None, None) == native.GP_ERR_INVALID


def test_row_plan_admits_repeated_destinations():
    """A repeated destination (cache rows {5, 9, 5, 2}: the reference's range
    check admits such sets, clientlib-viter.cpp:869-873) is no longer refused:
    the plan puts the second occurrence in a repeat layer, which needs device
    memory, so without a device creation fails on the allocation, not on the
    index.  The GPU test test_row_plan_repeated_destinations checks the sums
    against the oracle's sequential order."""
    import numpy as np
    idx = np.stack([np.arange(4), np.array([5, 9, 5, 2])], 1)
    rc, h = _plan(idx)
    msg = native.lib().gp_last_error()
    assert b"repeat" not in msg
    if rc == 0:  # a device is present
        layers, rows = ctypes.c_size_t(), ctypes.c_size_t()
        assert native.lib().gp_row_plan_repeats(h, ctypes.byref(layers), ctypes.byref(rows)) == 0
        assert (layers.value, rows.value) == (1, 1)
        native.lib().gp_row_plan_destroy(h)
    else:
        assert rc == native.GP_ERR_HIP and not h.value
    L = native.lib()
    assert L.gp_row_plan_repeats(None, None, None) == native.GP_ERR_INVALID
    assert L.gp_row_plan_create(None, None, 0, native.DoubleIndex(0, 0), 128, 0) == 1
    h = ctypes.c_void_p()
    assert L.gp_row_plan_create(ctypes.byref(h), None, 4, native.DoubleIndex(0, 0), 128, 0) == 1
    assert L.gp_scatter_add_rows_planned(None, None, None, None) == 1


def test_launch_plans_stable_while_device_is_set_concurrently():
    """The CU count behind every launch plan is cached per device and never
    reset (gp_set_device used to zero a process-global that
    other threads were sizing grids from).  Several threads plan sums while
    another keeps calling gp_set_device; every plan must equal the one made
    before.  (ctypes releases the GIL during each call, so the calls overlap.)"""
    import threading
    L = native.lib()

    def plan(n, nb):
        a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        assert L.gp_bucket_sum_sweep_plan(n, nb, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)) == 0
        return a.value, b.value, c.value

    cases = [((1 << 30) + 7, 8), ((1 << 28) + 5, 2), (100 << 20, 3), (30 << 18, 5)]
    want = {k: plan(*k) for k in cases}
    stop = threading.Event()
    bad = []

    def planner():
        while not stop.is_set():
            for k in cases:
                if plan(*k) != want[k]:
                    bad.append(k)

    def setter():
        while not stop.is_set():
            L.gp_set_device(0)  # fails without a GPU; must never disturb the plans

    ts = [threading.Thread(target=planner) for _ in range(4)] + [threading.Thread(target=setter)]
    for t in ts:
        t.start()
    import time
    time.sleep(1.0)
    stop.set()
    for t in ts:
        t.join()
    assert not bad
    assert want[cases[0]][2] > 0  # the 4-GiB 8-way shard takes sweep chunks


def test_c_abi_consumer_builds_as_c99(tmp_path):
    """include/gp_reduce.h is a plain C header: tests/apps/c_abi_check.c, a C99
    consumer of the C-ABI, compiles with -pedantic -Werror and links against the
    product library with gcc (no HIP or C++ types needed).  Run without a GPU it
    exercises the error convention (GP_ERR_INVALID + gp_last_error) from C, then
    stops at the device count; tests/test_gpu_parity.py runs it whole."""
    exe = tmp_path / "c_abi_check"
    oracle_dir = os.path.join(REPO, "oracle", "build")
    subprocess.run(["gcc", "-std=c99", "-pedantic", "-Wall", "-Wextra", "-Werror", "-O2",
                    "-I", os.path.join(REPO, "include"),
                    os.path.join(REPO, "tests", "apps", "c_abi_check.c"), "-o", str(exe),
                    "-L", os.path.dirname(native.LIB_PATH), "-lgp_reduce", "-L", oracle_dir, "-loracle",
                    f"-Wl,-rpath,{os.path.dirname(native.LIB_PATH)}:{oracle_dir}",
                    "-Wl,-rpath-link,/opt/rocm/lib"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert "error convention: GP_ERR_INVALID + gp_last_error() ok" in r.stdout, r.stdout + r.stderr
    if r.returncode != 0:  # no GPU here: the device count fails loudly, nothing falls back
        assert r.returncode == 1 and "gp_device_count" in r.stderr, r.stdout + r.stderr
    else:
        assert "c_abi_check ok" in r.stdout


def test_sweep_shapes_and_plan_cover_every_headline_shard():
    """For 1-8 buckets and the 1/2/4/8-GPU shards of the 1M x 1024 table, the
    launch plan uses the documented sweep shapes (gp_kernels.hpp SweepShape:
    32-KiB tiles, bursts of 1 at 2-8 buckets; 16-KiB tiles, bursts of 8 at 1)
    and its chunks never overrun the shard (96-MiB chunks, then 64-MiB ones at
    3-8 buckets, on 256 CUs without a device)."""
    L = native.lib()
    sp = native.SumPlan()
    for shards in (1, 2, 4, 8):
        n = (1 << 30) // shards  # floats per shard
        for nb in range(1, 9):
            assert L.gp_bucket_sum_launch_plan(n, nb, ctypes.byref(sp)) == 0
            assert sp.sweep_launches >= 3, (shards, nb)
            if nb == 1:
                assert (sp.sweep_reg_tiles, sp.sweep_burst_tiles, sp.sweep_tile_kib) == (14, 8, 16)
            else:
                assert (sp.sweep_reg_tiles, sp.sweep_burst_tiles, sp.sweep_tile_kib) == (7, 1, 32)
            big = (160 + sp.sweep_reg_tiles * sp.sweep_tile_kib) * 1024 * 256  # bytes per 96-MiB chunk
            assert big == 96 << 20
            small = (160 + 6 * 16) * 1024 * 256 if sp.small_sweep_launches else 0
            if nb <= 2:
                assert sp.small_sweep_launches == 0
            covered = sp.sweep_launches * big + sp.small_sweep_launches * small
            assert covered <= 4 * n and 4 * n - covered < big, (shards, nb, covered)
