"""Benchmark of the GeePS gradient-update reduction path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...)

Workload (BASELINE.json north-star target: the 8-way sum at 1M x 1024; at N = 8
it is configs[2]'s shape): a 1M-row x 1024 fp32 parameter table, 8 synthetic
clients, the table row-range sharded over the N GPUs as N server shards
(src/client/clientlib-viter.cpp:674-682).  Client c is
hosted on rank c % N; its delta buffer is uniform in [-0.5, 0.5) (seed 1000+c).

A *step* is one device-resident N-way reduction: each shard adds the 8 client
buckets for its rows into its master copy in client order 0..7 with one
gp_bucket_sum_apply call (the reference's TabletStorage::apply_updates x 8,
src/server/tablet-server.cpp:119-134); for a 4 GiB shard that call issues 42
launches of the phase-separated sweep kernel, each summing a 96-MiB chunk of
the shard, and one for the last 64 MiB (gp_bucket_sum_launch_plan gives every
launch by form).  At N > 1 the buckets were first moved
to their shard by RCCL all-to-all (untimed here; the exchange-inclusive step
exchange + apply + all-gather refresh is timed separately and reported as
`exchange_inclusive`).  Total work is fixed as N grows: scaling "strong".

value = gradient (delta) bytes reduced per second, whole job:
        clients * rows * width * 4 B / max-over-ranks step time.
roofline.traffic = HBM bytes per launch of the dominant kernel from two
        rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over this bench's
        headline step in child processes, measured in this run at N = 1
        (profiles/pmc_traffic.json's committed value otherwise, and beside it).
roofline.achieved = algorithmic HBM bytes of one step ((clients + 2) * shard
        bytes: 8 bucket reads + master read + master write) / the step's
        average kernel time from HIP events around its launches on their
        stream; per launch, the same ratio (avg_launch_ms is what rocprofv3
        reports for the kernel).
cpu_baseline = the oracle's restatement of the reference server arithmetic
        (sequential vsAdd per client, gcc -O3) on rank 0's host cores, on the
        full 1M x 1024 table with the same 8 clients: 1 thread, plus the
        process's CPU share (OMP_NUM_THREADS) as "all_cores".
Other legs at N = 1 (rank 0): config2 (BASELINE configs[1], 2 clients),
client_rowops (scatter-add / fused init / gather of the table's 8M RowData
rows, random and identity DoubleIndex, unplanned and through a row plan),
host_inclusive (pinned H2D + sum + D2H, serialized and pipelined, full table),
libgeeps_clock (the drop-in library's clock through include/geeps.hpp, 1 and
2 processes on the same 4 GiB table), per_rank_emulation (each N-GPU rank's
shard sum timed on this GPU, emulated: true).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip table)
METRIC = "GB/s gradient rows reduced (device-resident N-way fp32 sum); % HBM roofline"
def sum_launch_plan(num_vals: int, num_buckets: int) -> dict:
    """The dominant kernel of one N-way sum of num_vals floats and how many
    launches of it one sum issues, from the library's own launch plan
    (gp_bucket_sum_launch_plan).  Shards of at least 3 whole 96-MiB chunks go
    to bucket_sum_sweep_kernel<NB, 7, 1, false, 8> at 2-8 buckets (7 register
    tiles of 32 KiB, bursts of 1), <1, 14, 8, false, 4> at 1 (the 4 GiB
    headline shard: 42 of them), then whole 64-MiB chunks to
    bucket_sum_sweep_kernel<NB, 6, 4> (the
    4 GiB shard: 1), the rest to the tile-major bucket_sum_phased_kernel and
    the mixed / scalar forms; smaller shards start at the 64-MiB sweep or the
    phased kernel.  `launches` counts the dominant kernel only and `share` is
    its part of the shard, so a per-launch time or byte figure (call time x
    share / launches) compares with rocprofv3's average for that kernel;
    `kernel_id` names the instantiation as rocprofv3 prints it (buckets,
    register tiles, burst depth)."""
    import ctypes
    from geeps_amd import native
    p = native.SumPlan()
    native.check(native.lib().gp_bucket_sum_launch_plan(num_vals, num_buckets, ctypes.byref(p)),
                 "gp_bucket_sum_launch_plan")
    cus = torch.cuda.get_device_properties(0).multi_processor_count if torch.cuda.is_available() else 256
    # (kernel, launches, register tiles, tiles per burst, KiB per tile)
    forms = [("bucket_sum_sweep_kernel", p.sweep_launches, p.sweep_reg_tiles, p.sweep_burst_tiles,
              p.sweep_tile_kib),
             ("bucket_sum_sweep_kernel", p.small_sweep_launches, 6, p.small_sweep_burst_tiles, 16),
             ("bucket_sum_phased_kernel", p.phased_launches, p.phased_reg_tiles, None, 16)]
    total = p.sweep_launches + p.small_sweep_launches + p.phased_launches + p.other_launches
    for kernel, n, rt, tg, kib in forms:
        if n > 0:
            share = 1.0
            if kernel == "bucket_sum_sweep_kernel":  # 160 KiB of LDS + rt register tiles per CU
                share = min(1.0, n * (160 + rt * kib) * 1024 // 4 * cus / num_vals)
            kid = f"{kernel}<{num_buckets}, {rt}, {tg}," if tg else f"{kernel}<{num_buckets}, {rt},"
            return {"kernel": kernel, "kernel_id": kid, "launches": n,
                    "other_launches": total - n, "reg_tiles": rt, "burst_tiles": tg, "share": share}
    return {"kernel": "bucket_sum_vec_kernel", "kernel_id": f"bucket_sum_vec_kernel<{num_buckets},",
            "launches": 1, "other_launches": total - 1, "reg_tiles": None, "share": 1.0}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--rows", type=int, default=1 << 20)
    p.add_argument("--width", type=int, default=1024)
    p.add_argument("--clients", type=int, default=8)
    p.add_argument("--exchange", choices=["a2a", "rs"], default="a2a")
    p.add_argument("--exchange-steps", type=int, default=5)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-host-inclusive", action="store_true")
    p.add_argument("--cpu-rows", type=int, default=1 << 20)
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--no-rowops", action="store_true")
    p.add_argument("--rowops-only", nargs="*", default=None, choices=list(ROWOP_LEGS),
                   help="run only these client row-op legs (PMC passes)")
    p.add_argument("--rowops-index", nargs="*", default=["random", "identity"],
                   choices=["random", "identity"], help="DoubleIndex kinds of the row-op legs")
    p.add_argument("--no-config2", action="store_true")
    p.add_argument("--no-per-rank", action="store_true",
                   help="skip the one-GPU emulation of the N-GPU runs' per-rank work")
    p.add_argument("--no-e2e", action="store_true",
                   help="skip the libgeeps end-to-end clock legs")
    p.add_argument("--no-multi-e2e", action="store_true",
                   help="at N > 1, skip the libgeeps one-process-per-GPU leg")
    p.add_argument("--no-hbm-probe", action="store_true")
    p.add_argument("--no-separate-alloc", action="store_true",
                   help="skip timing the headline sum on separately allocated buffers")
    p.add_argument("--no-pmc", action="store_true",
                   help="skip the in-run PMC traffic passes (roofline.traffic then comes from "
                        "profiles/pmc_traffic.json)")
    p.add_argument("--layout", choices=["arena", "separate"], default="arena",
                   help="HBM layout of buckets + master: one arena (master last) or one "
                        "allocation per buffer")
    return p.parse_args(argv)


def init_dist(n_gpus, backend="nccl"):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != n_gpus:
        raise SystemExit(f"--gpus {n_gpus} but WORLD_SIZE={world}")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend == "gloo":  # CPU rehearsal of the multi-rank flow (tests only)
        if world > 1:
            dist.init_process_group("gloo")
        return (dist.get_rank() if world > 1 else 0), world, torch.device("cpu")
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return (dist.get_rank() if world > 1 else 0), world, torch.device("cuda", local)


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize()


def barrier(world, dev):
    if world > 1:
        dist.barrier()
    _sync(dev)


def max_over_ranks(x: float, world: int, dev) -> float:
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def make_deltas(hosted, n, dev, layout="arena", extra=0):
    """The hosted clients' delta buffers.  With layout "arena" they are carved
    from one allocation followed by `extra` floats (the master shard at N = 1),
    returned as the last element; with "separate" each is its own allocation."""
    g = torch.Generator(device=dev)
    arena = None
    if layout == "arena":
        arena = torch.empty(len(hosted) * n + extra, dtype=torch.float32, device=dev)
    out = []
    for j, c in enumerate(hosted):
        g.manual_seed(1000 + c)
        if arena is not None:
            d = arena[j * n:(j + 1) * n]
            torch.rand(n, generator=g, device=dev, out=d)
        else:
            d = torch.rand(n, generator=g, device=dev)
        d.sub_(0.5)
        out.append(d)
    tail = arena[len(hosted) * n:] if (arena is not None and extra) else None
    return out, tail


def timed_apply(red, steps, warmup, world, dev):
    """Device-resident reduction: K launches, HIP events around each one on the
    launch stream, wall clock bracketed by barrier + synchronize."""
    for _ in range(warmup):
        red.apply()
    if dev.type != "cuda":  # CPU rehearsal: wall clock only
        barrier(world, dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            red.apply()
        barrier(world, dev)
        wall = time.perf_counter() - t0
        return wall, [wall * 1e3 / steps] * steps
    stream = torch.cuda.current_stream()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(steps)]
    barrier(world, dev)
    t0 = time.perf_counter()
    for a, b in evs:
        a.record(stream)
        red.apply()
        b.record(stream)
    torch.cuda.synchronize()
    barrier(world, dev)
    wall = time.perf_counter() - t0
    kernel_ms = [a.elapsed_time(b) for a, b in evs]
    return wall, kernel_ms


def hbm_probe(src, dst, reps=5):
    """Same-box HBM context for every kernel's roofline.frac, timed with HIP
    events on the launch stream over one 4 GiB bucket:
      read   gp_hbm_probe(GP_PROBE_READ): the buffer streamed once, read-only
      write  gp_hbm_probe(GP_PROBE_WRITE): written once (the runtime's fill)
      copy   gp_memcpy_async D2D (hipMemcpyAsync: 1 read + 1 write stream)
    each the fastest shape found for that stream alone.  A kernel reading R and
    writing W bytes is then modelled as R / read_rate + W / write_rate
    (`model_ms`): a best case, since it charges nothing for mixing reads and
    writes on HBM, and HBM boxes differ by several percent."""
    from geeps_amd import native
    lib = native.lib()
    stream = torch.cuda.current_stream()
    nbytes = src.numel() * src.element_size()

    def timed(fn):
        fn()
        ms = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            fn()
            b.record(stream)
            b.synchronize()
            ms.append(a.elapsed_time(b))
        return sum(ms) / len(ms)

    t_copy = timed(lambda: native.check(lib.gp_memcpy_async(dst.data_ptr(), src.data_ptr(), nbytes,
                                                            stream.cuda_stream), "gp_memcpy_async"))
    t_read = timed(lambda: native.check(lib.gp_hbm_probe(0, src.data_ptr(), src.numel(),
                                                         stream.cuda_stream), "gp_hbm_probe"))
    t_write = timed(lambda: native.check(lib.gp_hbm_probe(1, dst.data_ptr(), dst.numel(),
                                                          stream.cuda_stream), "gp_hbm_probe"))
    return {"read_GBps": round(nbytes / (t_read / 1e3) / 1e9, 1),
            "write_GBps": round(nbytes / (t_write / 1e3) / 1e9, 1),
            "copy_GBps": round(2 * nbytes / (t_copy / 1e3) / 1e9, 1), "bytes": nbytes,
            "read_ms": round(t_read, 4), "write_ms": round(t_write, 4), "copy_ms": round(t_copy, 4),
            "note": "one 4 GiB buffer: read-only and write-only streams (gp_hbm_probe) and a "
                    "hipMemcpyAsync D2D copy, on this box"}


def model_ms(read_bytes, write_bytes, probe):
    """The same box's two-rate HBM model of a kernel's bytes (hbm_probe)."""
    if not probe:
        return None
    return read_bytes / (probe["read_GBps"] * 1e9) * 1e3 + write_bytes / (probe["write_GBps"] * 1e9) * 1e3


def regen_delta(c, n, dev):
    """Client c's delta buffer regenerated: the same values make_deltas wrote."""
    g = torch.Generator(device=dev)
    g.manual_seed(1000 + c)
    d = torch.rand(n, generator=g, device=dev)
    d.sub_(0.5)
    return d


# Per element of a reduce-scatter exchange's refreshed table against the
# client-order sum: |err| <= clients ulps of the largest partial sum
# (tests/test_shard_gloo.py writes the same bound, steps = 1 here).
def rs_tolerance(clients):
    import numpy as np
    return clients * float(np.finfo(np.float32).eps) * (0.5 * clients + 1)


def exchange_check(red, deltas, R, W, C, dev, world, kind):
    """configs[2]'s parity check on the ranks themselves: one
    clean clock -- push (the RCCL exchange) -> apply (the HIP N-way sum) ->
    refresh (all-gather) -- on a zeroed master, then on EVERY rank the
    refreshed full table against
      * the client-order sum ((0 + d0) + d1) + ... + d{C-1} of all C seeded
        deltas regenerated on this rank's device, every element (the reference
        server applies the clients' messages in arrival order,
        tablet-server.cpp:119-134; a2a: bit-exact, rs: rs_tolerance);
      * a numpy restatement of that sum on sampled rows: row 0, the last row,
        the first and last row of every shard (the a2a split offsets and the
        all-gather's padded-shard unpacking of an uneven partition) and 8
        seeded random rows.
    Returns {"ok", "max_abs_err", "rows_sampled", ...}, reduced over ranks
    (ok: all ranks; max_abs_err: the largest)."""
    import numpy as np
    L = red.layout
    red.master.zero_()
    table = red.step(deltas)[:R * W]
    _sync(dev)
    rows = {0, R - 1}
    for s, c in zip(L.starts, L.counts):
        if c:
            rows.update((s, s + c - 1))
    rows.update(int(r) for r in np.random.default_rng(7).integers(0, R, 8))
    rows = sorted(rows)
    idx = torch.tensor(rows, dtype=torch.long, device=dev)
    exp = torch.zeros(R * W, dtype=torch.float32, device=dev)
    sampled = np.zeros((C, len(rows), W), np.float32)
    for c in range(C):
        d = regen_delta(c, R * W, dev)
        exp.add_(d)
        sampled[c] = d.view(R, W).index_select(0, idx).cpu().numpy()
        del d
    m = np.zeros((len(rows), W), np.float32)
    for c in range(C):  # fp32 adds in client order
        m = m + sampled[c]
    got = table.view(R, W).index_select(0, idx).cpu().numpy()
    bits_equal = torch.equal(table.view(torch.int32), exp.view(torch.int32))
    err = float(exp.sub_(table).abs_().max().item()) if R * W else 0.0  # (in place: no 4-GiB temporaries)
    err_rows = float(np.abs(got - m).max()) if m.size else 0.0
    if kind == "a2a":
        ok = bits_equal and np.array_equal(got.view(np.uint32), m.view(np.uint32))
    else:
        ok = err <= rs_tolerance(C) and err_rows <= rs_tolerance(C)
    del exp
    flag = -max_over_ranks(-(1.0 if ok else 0.0), world, dev)  # min over ranks
    return {"ok": flag == 1.0, "max_abs_err": max_over_ranks(max(err, err_rows), world, dev),
            "bar": "bit-exact vs client order" if kind == "a2a" else f"|err| <= {rs_tolerance(C):.3g}",
            "rows_sampled": len(rows), "elements_checked": R * W, "ranks": world}


def timed_exchange(red, deltas, steps, warmup, world, dev):
    for _ in range(warmup):
        red.step(deltas)
    barrier(world, dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        red.step(deltas)
    barrier(world, dev)
    return time.perf_counter() - t0


def host_inclusive(rows, W, clients, dev, chunk_rows=16384, steps=2):
    """The path starts and ends in host memory: the client buckets arrive in
    pinned host buffers (as from the socket, clientlib-data.cpp:473-476), the
    refreshed shard leaves to one (recv_row_batch_gpu's H2D is its mirror,
    :128-130).  Full table (rows x W fp32, `clients` buckets), master resident
    in HBM.  Three schedules, each timed over `steps` steps after a warm-up:
      serialized  all H2D, then the N-way sum, then the D2H of the shard;
      pipelined   rows cut into chunks: H2D of chunk i (copy stream), the sum
                  of chunk i-1 (compute stream), the D2H of chunk i-2 (a third
                  stream), 3 device slots of `clients` chunk buffers;
      copy_bound  the pipelined schedule without the sum: what pinned PCIe
                  moves in this run, both directions at once."""
    from geeps_amd import rowops
    n = rows * W
    cn = chunk_rows * W
    nchunks = (rows + chunk_rows - 1) // chunk_rows
    host = [torch.empty(n, dtype=torch.float32, pin_memory=True) for _ in range(clients)]
    g = torch.Generator(device=dev)
    for c, h in enumerate(host):  # synthetic deltas made on the device, copied out once
        g.manual_seed(1000 + c)
        h.copy_(torch.rand(n, generator=g, device=dev).sub_(0.5))
    out = torch.empty(n, dtype=torch.float32, pin_memory=True)
    master = torch.zeros(n, dtype=torch.float32, device=dev)
    comp = torch.cuda.current_stream()
    s_in, s_out = torch.cuda.Stream(), torch.cuda.Stream()
    res = {"rows": rows, "width": W, "clients": clients, "chunk_rows": chunk_rows,
           "bytes_h2d": clients * n * 4, "bytes_d2h": n * 4}

    def timed(step):
        step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps

    # serialized: every bucket resident first
    dbuf = [torch.empty(n, dtype=torch.float32, device=dev) for _ in range(clients)]

    def serialized():
        with torch.cuda.stream(s_in):
            for h, d in zip(host, dbuf):
                d.copy_(h, non_blocking=True)
        comp.wait_stream(s_in)
        rowops.bucket_sum_apply(master, dbuf)
        s_out.wait_stream(comp)
        with torch.cuda.stream(s_out):
            out.copy_(master, non_blocking=True)
        comp.wait_stream(s_out)

    t_ser = timed(serialized)
    del dbuf
    torch.cuda.empty_cache()
    slots = [[torch.empty(cn, dtype=torch.float32, device=dev) for _ in range(clients)]
             for _ in range(3)]
    free = [torch.cuda.Event() for _ in range(3)]    # slot k no longer read by a sum
    landed = [torch.cuda.Event() for _ in range(3)]  # slot k's H2D done
    summed = [torch.cuda.Event() for _ in range(3)]  # chunk j's sum done (j % 3)
    for e in free:
        e.record(comp)

    def pipelined(with_sum=True):
        for i in range(nchunks + 2):
            if i < nchunks:  # H2D of chunk i into slot i % 3
                a, b = i * cn, min(n, (i + 1) * cn)
                s_in.wait_event(free[i % 3])
                with torch.cuda.stream(s_in):
                    for h, d in zip(host, slots[i % 3]):
                        d[:b - a].copy_(h[a:b], non_blocking=True)
                landed[i % 3].record(s_in)
            if 1 <= i <= nchunks:  # sum of chunk i - 1
                j = i - 1
                a, b = j * cn, min(n, (j + 1) * cn)
                comp.wait_event(landed[j % 3])
                if with_sum:
                    rowops.bucket_sum_apply(master[a:b], [d[:b - a] for d in slots[j % 3]])
                free[j % 3].record(comp)
                summed[j % 3].record(comp)
            if i >= 2:  # D2H of chunk i - 2
                j = i - 2
                a, b = j * cn, min(n, (j + 1) * cn)
                s_out.wait_event(summed[j % 3])
                with torch.cuda.stream(s_out):
                    out[a:b].copy_(master[a:b], non_blocking=True)
        comp.wait_stream(s_out)

    t_pipe = timed(pipelined)
    t_copy = timed(lambda: pipelined(False))
    delta = clients * n * 4
    for name, t in (("serialized", t_ser), ("pipelined", t_pipe), ("copy_bound", t_copy)):
        res[name] = {"ms_per_step": round(t * 1e3, 2), "delta_GBps": round(delta / t / 1e9, 2),
                     "pcie_GBps": round((clients + 1) * n * 4 / t / 1e9, 2)}
    res["pipelined_vs_copy_bound"] = round(t_copy / t_pipe, 4)
    res["note"] = ("pinned H2D of every client bucket + device N-way sum + D2H of the shard; "
                   "delta_GBps = client delta bytes / step time")
    del host, out, master, slots
    torch.cuda.empty_cache()
    return res


ROWOP_LEGS = ("scatter_add", "scatter_add_planned", "scatter_init", "scatter_init_planned",
              "gather", "gather_planned")


def _time_calls(fn, reps, stream, warmup=True):
    if warmup:
        fn()
    ms = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        fn()
        b.record(stream)
        b.synchronize()
        ms.append(a.elapsed_time(b))
    return sum(ms) / len(ms)


def rowops_leg(rows, W, dev, reps=5, indexes=("random", "identity"), only=None, probe=None):
    """The client half of the path at the same table size: the 1M x 1024 table
    through the 128-float API is R = 8M RowData rows.  Per DoubleIndex
    (random permutation of the destinations, and identity -- libgeeps' cache
    rows are in first-access order, so its real indexes are long runs):
      scatter_add          gp_scatter_add_rows: index read on device every call
                           (reference add_rows_from_double_index_gpu, row-op-util.cu:109-142)
      scatter_add_planned  the same through a gp_row_plan (what libgeeps runs)
      scatter_init         gp_scatter_init_rows: fused zerofy + add (common-util.hpp:445-456 + a3)
      scatter_init_planned the same through the plan
      gather               gp_gather_rows (assign_rows_to_double_index_gpu, :39-72)
      gather_planned       the same through a gather plan (what libgeeps' Read runs)
    Algorithmic bytes per call: add 3*R*512, init / gather 2*R*512, plus the
    16-B DoubleIndex entries the kernel reads (every row unplanned; a plan's
    residual rows planned -- its dense runs read no index)."""
    from geeps_amd import native, rowops
    R = rows * W // 128
    stream = torch.cuda.current_stream()
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    x = torch.rand(R * 128, generator=g, device=dev)
    y = torch.zeros(R * 128, device=dev)
    out = {}
    if "random" in indexes and not only:
        # one throwaway index through the plan cache's first and second calls:
        # the process's first radix sort loads hipCUB's kernels and grows the
        # stream-ordered pool (one-time costs, ~5 ms), which would otherwise
        # land in the first leg's `second_call_ms`
        warm = torch.stack([torch.arange(R, device=dev), torch.randperm(R, generator=g, device=dev)], 1)
        for _ in range(2):
            rowops.add_rows_from_double_index_gpu(y, x, warm, R, (0, 0), 128, R * 128, validate=False)
        torch.cuda.synchronize()
        native.check(native.lib().gp_unplanned_cache_clear(), "gp_unplanned_cache_clear")
        del warm
    for kind in indexes:
        if kind == "random":
            dst = torch.randperm(R, generator=g, device=dev)
        else:
            dst = torch.arange(R, device=dev)
        idx = torch.stack([torch.arange(R, device=dev), dst], 1).contiguous()
        plan = rowops.RowPlan(idx, R, (0, 0), 128, R * 128)
        gplan = rowops.RowPlan(idx, R, (0, 0), 128, R * 128, kind="gather")
        info = plan.info()
        ginfo = gplan.info()
        legs = {}
        for name in ROWOP_LEGS:
            if only and name not in only:
                continue
            planned = name.endswith("_planned")
            pinfo = ginfo if name.startswith("gather") else info
            # dense runs read no index; residual rows (and unplanned calls) do
            index_rows = pinfo["rows"] - pinfo["dense_rows"] if planned else R
            nbytes = (3 if name.startswith("scatter_add") else 2) * R * 512 + 16 * index_rows
            writes = R * 512
            launches, other, share, kernel_id = 1, 0, 1.0, None
            # the unplanned calls plan themselves on the device (gp_reduce.h,
            # ABI 10-12): the first call with an index (`first_call_ms`) scans
            # it (one stream sync, as the reference's call syncs too), runs
            # its dense runs through the sweep forms and the rest through the
            # row kernels -- a scatter's unsorted rest through an inverse map
            # it builds -- and keeps the plan; later calls (`second_call_ms`,
            # `avg_ms`: the reference reusing each op's DoubleIndex every
            # clock) run it behind the device check, with no host round trip.
            # `plan_stats`: gp_unplanned_stats_get over this leg's calls.
            scan = "index_verify_kernel + "
            if name == "scatter_add":
                fn = lambda: rowops.add_rows_from_double_index_gpu(y, x, idx, R, (0, 0), 128, R * 128,
                                                                   validate=False)
                kernel = scan + ("bucket_sum_sweep_kernel" if kind == "identity"
                                 else "row_wave_kernel (the kept inverse map)")
            elif name == "scatter_init":
                fn = lambda: rowops.init_rows_from_double_index_gpu(y, x, idx, R, (0, 0), 128, R * 128,
                                                                    validate=False)
                kernel = scan + ("bucket_sum_sweep_kernel" if kind == "identity"
                                 else "row_wave_kernel (the kept inverse map)")
            elif name == "gather":
                fn = lambda: rowops.assign_rows_to_double_index_gpu(x, y, idx, R, (0, 0), 128, R * 128,
                                                                    validate=False)
                kernel = scan + ("bucket_sum_sweep_kernel" if kind == "identity" else "row_wave_kernel")
            elif name == "gather_planned":
                fn = lambda: gplan.gather(x, y)
                if ginfo["dense_rows"] == R:  # one dense run: the no-bucket sweep copy
                    pl = gplan.launches()
                    kernel = "bucket_sum_sweep_kernel" if pl["sweep"] else "bucket_sum_phased_kernel"
                    kernel_id = "bucket_sum_sweep_kernel<0, 6, 4, false," if pl["sweep"] else None
                    launches = pl["sweep"] or pl["phased"]
                    other = pl["phased"] + pl["other"] if pl["sweep"] else pl["other"]
                    cus = torch.cuda.get_device_properties(dev).multi_processor_count
                    share = min(1.0, pl["sweep"] * 16 * cus * 4096 / (R * 128)) if pl["sweep"] else 1.0
                else:
                    kernel = "row_wave_kernel"
            else:
                init = name == "scatter_init_planned"
                fn = (lambda: plan.init(y, x)) if init else (lambda: plan.add(y, x))
                if info["dense_rows"] == R:  # one dense run: the 1-bucket sum (init: zero-input form)
                    if init:  # one sweep shape (64-MiB chunks), then the tile-major rest
                        pl = plan.launches(True)
                        kernel = "bucket_sum_sweep_kernel" if pl["sweep"] else "bucket_sum_phased_kernel"
                        kernel_id = "bucket_sum_sweep_kernel<1, 6, 4, true," if pl["sweep"] else None
                        launches = pl["sweep"] or pl["phased"]
                        other = pl["phased"] + pl["other"] if pl["sweep"] else pl["other"]
                        cus = torch.cuda.get_device_properties(dev).multi_processor_count
                        share = min(1.0, pl["sweep"] * 16 * cus * 4096 / (R * 128)) if pl["sweep"] else 1.0
                    else:
                        sp = sum_launch_plan(R * 128, 1)
                        kernel, kernel_id = sp["kernel"], sp["kernel_id"]
                        launches, other, share = sp["launches"], sp["other_launches"], sp["share"]
                else:
                    kernel = "row_wave_kernel"
            first_ms = second_ms = None
            s0 = native.unplanned_stats()
            if not planned:  # the first and second calls with this index on their own
                native.check(native.lib().gp_unplanned_cache_clear(), "gp_unplanned_cache_clear")
                first_ms = _time_calls(fn, 1, stream, warmup=False)
                second_ms = _time_calls(fn, 1, stream, warmup=False)
            avg = _time_calls(fn, reps, stream)
            s1 = native.unplanned_stats()
            gbps = nbytes / (avg / 1e3) / 1e9
            leg = {"avg_ms": round(avg, 4), "GBps": round(gbps, 1),
                   "frac": round(gbps / HBM_PEAK_GBPS, 4), "bytes": nbytes, "kernel": kernel,
                   "launches": launches, "avg_launch_ms": round(avg * share / launches, 5)}
            if not planned:
                leg["plan_stats"] = {k: s1[k] - s0[k] for k in s1}
            if first_ms is not None:
                leg["first_call_ms"] = round(first_ms, 4)
                leg["first_call_frac"] = round(nbytes / (first_ms / 1e3) / 1e9 / HBM_PEAK_GBPS, 4)
                leg["second_call_ms"] = round(second_ms, 4)
            if other:  # the rest in other kernel forms; avg_launch_ms is the dominant one's share
                leg["other_launches"] = other
                leg["dominant_share"] = round(share, 6)
            mm = model_ms(nbytes - writes, writes, probe)
            if mm:
                leg["model_ms"] = round(mm, 4)
                leg["frac_of_model"] = round(mm / avg, 4)
            if planned:
                leg["plan"] = pinfo
            traffic = load_traffic(f"rowops_{name}_{kind}_r{R}_w128", kernel_id or kernel)
            if traffic:
                leg["traffic"] = traffic["bytes_per_launch"] * launches
                leg["traffic_source"] = traffic
            legs[name] = leg
        out[kind] = dict(rows=R, row_size=128, index=f"{kind} permutation of destinations"
                         if kind == "random" else "identity", **legs)
        plan.close()
        gplan.close()
        native.check(native.lib().gp_unplanned_cache_clear(), "gp_unplanned_cache_clear")
        del idx, dst
    return out


CPU_SHARE_PER_GPU = 16  # host threads per GPU on the pool's boxes (their per-GPU CPU share)


def cpu_threads() -> tuple[int, str]:
    """Threads for the all-cores CPU figure, and how they were chosen: the CPU
    share this process may use (OMP_NUM_THREADS when it grants more than one);
    otherwise the affinity mask capped at one GPU's share of the box
    (CPU_SHARE_PER_GPU: a 256-thread box hosts 8 GPUs and the harness sizes a
    one-GPU job at 16), so an environment that pins OMP_NUM_THREADS=1 still
    gets an all-cores figure, with its source stated."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = nproc
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 1:
        t = min(int(env), aff)
        return t, f"OMP_NUM_THREADS={env} (this process's CPU share; nproc={nproc}, affinity={aff})"
    t = min(aff, CPU_SHARE_PER_GPU)
    why = f"OMP_NUM_THREADS={env}" if env else "OMP_NUM_THREADS unset"
    return t, (f"{why}; affinity mask ({aff} of nproc={nproc}) capped at one GPU's CPU share "
               f"({CPU_SHARE_PER_GPU})")


def cpu_baseline(rows, W, clients, seconds):
    """The oracle's restatement of the reference server arithmetic (sequential
    vsAdd per client message, gcc -O3, oracle/oracle.c) timed on the host, on
    the FULL table: `clients` synthetic client buffers of rows x W fp32 and a
    master of the same size.  1 thread = the reference's one tablet-server
    thread per channel (src/client/clientlib.cpp:102-105); the all-cores
    figure splits rows over threads as num_comm_channels server threads do
    (clientlib.cpp:216-224)."""
    import numpy as np
    from oracle import oracle
    n = rows * W
    threads, how = cpu_threads()
    t0 = time.perf_counter()
    ups = [oracle.fill_uniform(np.empty(n, np.float32), 1000 + c, threads) for c in range(clients)]
    master = np.zeros(n, np.float32)
    oracle.apply_updates(master, ups, threads=threads)  # fault the pages in
    setup = time.perf_counter() - t0
    rounds, t0 = 0, time.perf_counter()
    while True:
        oracle.apply_updates(master, ups)
        rounds += 1
        dt = time.perf_counter() - t0
        if dt >= seconds or rounds >= 50:
            break
    per = dt / rounds
    res = {"value": clients * n * 4 / per / 1e9, "unit": "GB/s", "cores": 1, "kind": "port",
           "sample": f"full table: {rows} rows x {W} fp32, {clients} clients applied sequentially "
                     f"per message (oracle_apply_updates, gcc -O3), {rounds} rounds in {dt:.1f} s",
           "ms_per_round": round(per * 1e3, 1)}
    if threads > 1:
        t0, r2 = time.perf_counter(), 0
        while True:
            oracle.apply_updates(master, ups, threads=threads)
            r2 += 1
            dt2 = time.perf_counter() - t0
            if dt2 >= seconds / 2 or r2 >= 100:
                break
        per2 = dt2 / r2
        res["all_cores"] = {"value": clients * n * 4 / per2 / 1e9, "unit": "GB/s", "cores": threads,
                            "threads_from": how, "ms_per_round": round(per2 * 1e3, 1),
                            "note": "row range split over threads = num_comm_channels "
                                    "server threads (clientlib.cpp:216-224)"}
    else:
        res["all_cores_skipped"] = f"1 thread available ({how})"
    res["setup_s"] = round(setup, 1)
    try:
        with open("/proc/cpuinfo") as f:
            model = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), "")
        res["cpu_model"] = model
    except OSError:
        pass
    res["nproc"] = os.cpu_count()
    del ups, master
    return res


def load_traffic(workload_key, kernel):
    """PMC HBM bytes per launch of `kernel` for this workload, from
    profiles/pmc_traffic.json (written by scripts/pmc_traffic.py from separate
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this bench), with where
    it came from: {"bytes_per_launch", "kernel" (the name the counters were
    filtered on), "source", "emulated" (true: an N-GPU rank's work measured on
    one GPU), "round"}.  None when absent or measured on another kernel than
    the one this run launches."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            entry = json.load(f).get(workload_key)
        if entry is None or kernel not in entry.get("kernel", ""):
            return None
        return {"bytes_per_launch": float(entry["hbm_bytes_per_launch"]),
                "kernel": entry["kernel"], "source": f"profiles/pmc_traffic.json[{workload_key}]",
                "emulated": bool(entry.get("emulated", False)),
                "round": entry.get("round")}
    except (OSError, ValueError, KeyError):
        return None


def measure_traffic(rows, W, clients, kernel_id, timeout_s=150):
    """HBM traffic per launch of the headline kernel, measured in this run: two
    child processes, each this bench (headline step only, 2 steps + 1 warm-up)
    under `rocprofv3 --pmc <counter> --kernel-trace`, one counter per pass
    (FETCH_SIZE, then WRITE_SIZE), each under a hard time limit.  Per launch:
    2 * FETCH_SIZE + WRITE_SIZE (KiB), the gfx950 correction of
    MI355X_MICROARCH.md's HBM section, averaged over the dispatches of the
    instantiation `kernel_id` names.  Returns (result, None) or (None, reason);
    the caller falls back to profiles/pmc_traffic.json."""
    import csv
    import glob
    import shutil
    import statistics
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None, "rocprofv3 not found"
    child = [sys.executable, os.path.join(REPO, "bench.py"), "--rows", str(rows), "--width", str(W),
             "--clients", str(clients), "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
             "--no-host-inclusive", "--no-hbm-probe", "--no-config2", "--no-e2e", "--no-rowops",
             "--no-per-rank", "--no-pmc", "--no-separate-alloc"]
    kib = {}
    dispatches = {}
    with tempfile.TemporaryDirectory(prefix="geeps_pmc_") as tmp:
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            out = os.path.join(tmp, counter)
            cmd = ["timeout", "-s", "KILL", str(timeout_s), prof, "--pmc", counter, "--kernel-trace",
                   "--output-format", "csv", "-d", out, "-o", "run", "--"] + child
            r = subprocess.run(cmd, cwd=tmp, capture_output=True, text=True,
                               env=dict(os.environ, TMPDIR=tmp))
            if r.returncode != 0:
                return None, f"rocprofv3 --pmc {counter} exited {r.returncode}: {r.stderr[-300:]}"
            vals = []
            for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
                with open(f) as fh:
                    for row in csv.DictReader(fh):
                        if kernel_id in row["Kernel_Name"] and row["Counter_Name"] == counter:
                            vals.append(float(row["Counter_Value"]))
            if not vals:
                return None, f"no {counter} rows for {kernel_id!r}"
            kib[counter] = statistics.fmean(vals)
            dispatches[counter] = len(vals)
    hbm = 2 * kib["FETCH_SIZE"] * 1024 + kib["WRITE_SIZE"] * 1024
    return {"bytes_per_launch": hbm, "kernel": kernel_id, "dispatches": dispatches,
            "FETCH_SIZE_KiB_mean": round(kib["FETCH_SIZE"], 1),
            "WRITE_SIZE_KiB_mean": round(kib["WRITE_SIZE"], 1),
            "source": "measured in this run: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of "
                      "this bench's headline step in child processes (2 * FETCH + WRITE)",
            "emulated": False}, None


ALEXNET_ROWS = 476292  # tests/test_libgeeps.py ALEXNET_BLOBS, each blob padded to 128-float rows


def _clock_bench_module():
    import importlib.util
    path = os.path.join(REPO, "scripts", "run_clock_bench.py")
    spec = importlib.util.spec_from_file_location("run_clock_bench", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


# The two cross-GPU data paths of libgeeps: "staged" =
# a peer's oplog slice and a peer's refreshed shard each peer-copied over xGMI
# into local HBM once (the default across GPUs); "in_place" = the server's sum
# and the client's Reads load the peer's HBM directly over xGMI.
PEER_PATHS = {"staged": {"GEEPS_STAGE_PEER_UPDATES": "1", "GEEPS_STAGE_PEER_REFRESH": "1"},
              "in_place": {"GEEPS_STAGE_PEER_UPDATES": "0", "GEEPS_STAGE_PEER_REFRESH": "0"}}


def libgeeps_multi_gpu_leg(n_gpus, rows, W, clocks=5, warmup=2, alex_clocks=10, gpus_seen=None,
                           tables=("1Mx1024", "alexnet")):
    """configs[2] / configs[4] through the drop-in, one process per GPU: the
    clock bench (scripts/apps/geeps_clock_bench.cpp through include/geeps.hpp)
    as n_gpus worker + tablet-server processes, process p on GPU p % count
    (GEEPS_TEST_SPREAD_DEVICES=1), same-node IPC transport, for both
    cross-GPU data paths (PEER_PATHS), on two tables:
      1Mx1024  the bench's rows x W fp32 table as RowData rows, BSP
      alexnet  the AlexNet-sized table (configs[4]), staleness bound 1
    Each worker checks its last Read over every element (read_ok).  Rank 0 of
    `bench.py --gpus N` runs this before any rank opens a GPU; on a one-GPU box
    the same code runs every process on GPU 0 (a rehearsal: both switches
    forced, so the staged copies run as peer copies within one GPU)."""
    mod = _clock_bench_module()
    if not os.path.exists(mod.BIN):
        return {"skipped": f"{os.path.relpath(mod.BIN, REPO)} not built (__graft_entry__.build())"}
    rd_rows = rows * W // 128
    gpus = gpus_seen if gpus_seen is not None else torch.cuda.device_count()
    out = {"app": "scripts/apps/geeps_clock_bench.cpp", "processes": n_gpus, "gpus_seen": gpus,
           "one_process_per_gpu": gpus >= n_gpus, "transport": "ipc (same node)", "clocks": clocks,
           "warmup": warmup}
    base_env = {"GEEPS_TEST_SPREAD_DEVICES": "1"}
    if gpus >= n_gpus:  # one process per GPU: the default hardware queues
        base_env["CLOCK_BENCH_HW_QUEUES"] = os.environ.get("GPU_MAX_HW_QUEUES", "4")
    failed = None
    # the default cross-GPU path (staged) on both tables first, then in place;
    # the whole leg within a time budget, so the scaling runs it precedes stay
    # short (GEEPS_BENCH_MULTI_BUDGET_S, default 150 s)
    budget_s = float(os.environ.get("GEEPS_BENCH_MULTI_BUDGET_S", "150"))
    out["budget_s"] = budget_s
    t_leg = time.monotonic()
    runs = [(table, nrows, slack, ck, path, env)
            for path, env in PEER_PATHS.items()
            for table, nrows, slack, ck in (("1Mx1024", rd_rows, 0, clocks), ("alexnet", ALEXNET_ROWS, 1, alex_clocks))
            if table in tables]
    for table, nrows, slack, ck, path, env in runs:
        key = f"{table}_{path}"
        if failed:  # one failure (or hang) ends the leg: the headline must not wait on it
            out[key] = {"skipped": f"after {failed} failed"}
            continue
        left = budget_s - (time.monotonic() - t_leg)
        if left < 20:
            out[key] = {"skipped": f"the leg's {budget_s:.0f}-s budget is spent"}
            continue
        t_run = time.monotonic()
        try:
            r = mod.run(n_gpus, nrows, ck, warmup, slack, "ipc", timeout=max(20.0, min(150.0, left)),
                        extra_env=dict(base_env, **env))
        except Exception as exc:  # report it, skip the rest
            out[key] = {"error": f"{type(exc).__name__}: {str(exc)[-800:]}",
                        "wall_s": round(time.monotonic() - t_run, 1)}
            failed = key
            continue
        out[key] = {"rows": nrows, "slack": slack, "ms_per_clock": r["ms_per_clock_max"],
                    "wall_s": round(time.monotonic() - t_run, 1),
                    "delta_GBps": r["aggregate_delta_GBps"], "read_ok": r["read_ok"],
                    "read_checked": r["read_checked"], "devices": r["devices"],
                    "nr_peer_staged": r.get("nr_peer_staged"),
                    "nr_refresh_staged": r.get("nr_refresh_staged"),
                    "nr_refresh_in_place": r.get("nr_refresh_in_place")}
    out["wall_s"] = round(time.monotonic() - t_leg, 1)
    return out


# libgeeps' default across GPUs (GEEPS_STAGE_PEER_UPDATES / _REFRESH unset:
# client_net.cpp stages a peer on another GPU) and the noise band within which
# the default counts as no slower than the alternative.
DEFAULT_PEER_PATH = "staged"
PEER_PATH_BAND = 0.03


def multi_gpu_verdict(multi: dict, default: str = DEFAULT_PEER_PATH, band: float = PEER_PATH_BAND) -> dict:
    """Top-level scalars that settle libgeeps' cross-GPU default from one
    `bench.py --gpus N` record, per table of the leg:
      libgeeps_multi_gpu_<table>_<path>_ms_per_clock  both paths' clocks
      libgeeps_multi_gpu_<table>_faster_path           the faster one
      libgeeps_multi_gpu_<table>_default_ok            default <= other x (1 + band)
    and overall libgeeps_multi_gpu_default_ok (every table measured on both
    paths, with every Read exact, and the default no slower on each) and
    libgeeps_multi_gpu_default_path.  A table missing a path (skipped,
    failed, a Read not exact) makes default_ok null: not decided."""
    other = "in_place" if default == "staged" else "staged"
    out = {"libgeeps_multi_gpu_default_path": default}
    oks = []
    for table in ("1Mx1024", "alexnet"):
        ms = {}
        for path in (default, other):
            r = multi.get(f"{table}_{path}")
            if isinstance(r, dict) and "ms_per_clock" in r and r.get("read_ok"):
                ms[path] = float(r["ms_per_clock"])
                out[f"libgeeps_multi_gpu_{table}_{path}_ms_per_clock"] = ms[path]
        if len(ms) < 2:
            out[f"libgeeps_multi_gpu_{table}_default_ok"] = None
            oks.append(None)
            continue
        ok = ms[default] <= ms[other] * (1.0 + band)
        out[f"libgeeps_multi_gpu_{table}_faster_path"] = min(ms, key=ms.get)
        out[f"libgeeps_multi_gpu_{table}_default_ok"] = ok
        oks.append(ok)
    out["libgeeps_multi_gpu_default_ok"] = None if (not oks or None in oks) else all(oks)
    return out


def pre_gpu_multi_leg(args, backend):
    """At N > 1 (one rank per GPU under torch.distributed.run): rank 0 runs
    libgeeps_multi_gpu_leg across the N GPUs while the other ranks wait on a
    file store WITHOUT touching a GPU; nothing of the RCCL harness exists yet.
    Returns rank 0's result (None elsewhere and at N = 1)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1 or backend != "nccl" or args.no_e2e or args.no_multi_e2e:
        return None
    import datetime
    import tempfile
    rank = int(os.environ.get("RANK", "0"))
    # every rank of one torch.distributed.run has the same parent (the agent)
    path = os.path.join(tempfile.gettempdir(),
                        f"geeps_bench_{os.getppid()}_{os.environ.get('MASTER_PORT', '0')}")
    store = dist.FileStore(path, world)
    store.set_timeout(datetime.timedelta(seconds=1500))
    res = None
    if rank == 0:
        log(f"[rank 0] libgeeps one-process-per-GPU leg over {world} GPUs (before any rank opens a GPU)")
        try:
            res = libgeeps_multi_gpu_leg(world, args.rows, args.width)
        except Exception as exc:
            res = {"error": f"{type(exc).__name__}: {str(exc)[-500:]}"}
        store.set("libgeeps_leg_done", "1")
    else:
        store.wait(["libgeeps_leg_done"])
    return res


def libgeeps_leg(rows, W, clocks=10, warmup=5, procs=(1, 2)):
    """The drop-in path end to end: scripts/apps/geeps_clock_bench (built by
    __graft_entry__.build() against libgeeps.so and include/geeps.hpp, as an
    app links) run as P processes on this GPU, one GeePS worker + tablet server
    each, same-node IPC transport.  The table is the bench's rows x W fp32 as
    RowData rows (rows * W / 128 of them).  One clock = Read (gather from the
    segmented param cache) -> PreUpdate (the clock's oplog slice: direct
    oplog) -> device fill -> PostRead -> Update (no rows move) -> Clock (push,
    the server's bucket sum, the zero-copy refresh), through the public API.  P = 2 is configs[1]'s
    2 loopback clients; every worker updates every row each clock.
    delta_GBps = P * table bytes / the slowest worker's ms per clock."""
    mod = _clock_bench_module()
    if not os.path.exists(mod.BIN):
        return {"skipped": f"{os.path.relpath(mod.BIN, REPO)} not built (__graft_entry__.build())"}
    rd_rows = rows * W // 128
    out = {"app": "scripts/apps/geeps_clock_bench.cpp", "rows": rd_rows, "row_size": 128,
           "table_bytes": rd_rows * 512, "transport": "ipc (same node)", "clocks": clocks,
           "warmup": warmup}

    def leg(key, fn):
        # each run on its own: one that raises is recorded under its key and
        # the runs before it keep their numbers
        try:
            out[key] = fn()
        except Exception as exc:
            out[key] = {"error": f"{type(exc).__name__}: {str(exc)[-500:]}"}

    def run(P, env=None, rows=rd_rows, slack=0, transport="ipc", info=None, keep=()):
        r = mod.run(P, rows, clocks, warmup, slack, transport, timeout=120, extra_env=env)
        d = {"workers": P, "ms_per_clock": r["ms_per_clock_max"], "delta_GBps": r["aggregate_delta_GBps"]}
        if rows != rd_rows or slack:
            d.update(rows=rows, slack=slack)
        d.update(info or {})
        for k in keep:  # a result field, or (field, key to report it under)
            src, dst = (k, k) if isinstance(k, str) else k
            d[dst] = r.get(src)
        return d

    for P in procs:
        leg(f"p{P}", lambda P=P: run(P, keep=(("ms_per_clock", "ms_per_clock_each"),)))
    # the same clock with the direct oplog off: Update copies the app's rows
    # into the oplog (the fused init), as before round 3
    leg("p1_copy", lambda: run(1, {"GEEPS_DIRECT_OPLOG": "0"}, info={"direct_oplog": False}))
    # the same clock with direct reads (GEEPS_DIRECT_READ=1, opt-in: the app
    # treats Read buffers as read-only): Read hands out the in-place master
    # version's rows, so the gather's copy goes too.  A direct Read must lie in
    # one server's shard: at P = 2 the app declares one Read op per shard
    # (CLOCK_BENCH_READ_PER_SHARD=1, as per-blob ops mostly fall in one shard)
    direct = {"GEEPS_DIRECT_READ": "1", "CLOCK_BENCH_READ_PER_SHARD": "1"}
    dinfo = {"direct_read": True, "read_ops": "one per server shard"}
    for P in procs:
        leg(f"p{P}_direct_read", lambda P=P: run(P, direct, info=dinfo))
    # configs[4]'s shape: the AlexNet-sized table (60,965,224 parameters in
    # 476,292 RowData rows, blobs padded to whole rows) clocked by 8 worker
    # processes (8 server shards) sharing this GPU, staleness bound 1
    leg("p8_alexnet_slack1", lambda: run(8, None, ALEXNET_ROWS, 1, info={
        "note": "one table-wide op per clock; the per-blob op sequence is tests/test_libgeeps.py's "
                "configs[4] test"}))
    leg("p8_alexnet_slack1_direct_read", lambda: run(8, direct, ALEXNET_ROWS, 1, info=dinfo))
    # SURVEY §8(f)'s next rows, measured: read-my-writes (f#4: every refresh
    # re-applies the worker's own unpushed oplog, clientlib-data.cpp:132-150)
    # at configs[1]'s 2 processes, and the socket path other nodes take (f#2:
    # D2H of the oplog slice, ZMTP frames over loopback TCP, the server's H2D
    # and sum, the refresh back the same way) on the AlexNet-sized table
    leg("p2_read_my_writes", lambda: run(2, {"CLOCK_BENCH_RMW": "1"}, info={"read_my_writes": True},
                                         keep=("read_ok",)))

    def tcp():
        d = run(2, None, ALEXNET_ROWS, 0, "tcp", keep=("read_ok",),
                info={"transport": "ZMTP/3.0 over loopback TCP (the other-node path)"})
        moved = 2 * 2 * (ALEXNET_ROWS // 2) * 512  # each worker: its slice out, the peer shard back
        d["socket_GBps"] = round(moved / (d["ms_per_clock"] * 1e-3) / 1e9, 2)
        return d
    leg("p2_alexnet_tcp", tcp)
    # a4, the host tier: a gpu_memory_capacity that holds half of the
    # AlexNet-sized table's rows, so the other half lives in host memory
    # (vi_decide_param_cache); its Updates go device to host and are added on
    # the CPU, its pushes and refreshes carry [host rows][HBM rows], its Reads
    # gather on the host and copy up (clientlib-data.cpp:153-189, 280-344,
    # 398-434); 2 processes.  The peer server reads the host-tier rows from
    # the client's shared host oplog (nr_host_shared); `_frames`: with
    # GEEPS_HOST_SHARE=0 they travel in the socket frame instead
    host = {"CLOCK_BENCH_HOST_TIER_FRAC": "0.5"}

    def host_tier(env):
        d = run(2, env, ALEXNET_ROWS, 0, info={"host_tier_frac": 0.5},
                keep=("read_ok", "rows_host_tier", "nr_host_shared"))
        # the host rows cross PCIe four times a clock (Update down, the
        # server's staging up, the refresh down, Read up), every process's
        # over this one GPU's link here
        moved = 4 * d["rows_host_tier"] * 512
        d["pcie_bytes_per_clock"] = moved
        d["pcie_GBps"] = round(moved / (d["ms_per_clock"] * 1e-3) / 1e9, 2)
        return d
    leg("p2_alexnet_host_tier", lambda: host_tier(host))
    leg("p2_alexnet_host_tier_frames", lambda: host_tier(dict(host, GEEPS_HOST_SHARE="0")))
    return out


def per_rank_leg(deltas, master, rows, W, dev, ranks=(2, 4, 8), reps=10):
    """The per-rank work of the N-GPU runs, timed on this one GPU (emulated:
    true): at N GPUs each rank sums the 8 client buckets into a shard of
    rows / N rows (the exchange that moved them there is not in the step).
    Here the shard is the leading rows / N rows of the resident buckets and
    master, so no new allocation; `predicted_speedup` = the N = 1 step time
    (this run's headline kernel time) / the rank's time.  DESIGN.md §7."""
    from geeps_amd import rowops
    stream = torch.cuda.current_stream()
    out = {}
    for N in ranks:
        n = (rows // N) * W
        bk = [d[:n] for d in deltas]
        m = master[:n]
        avg = _time_calls(lambda: rowops.bucket_sum_apply(m, bk), reps, stream)
        plan = sum_launch_plan(n, len(bk))
        gbps = (len(bk) + 2) * n * 4 / (avg / 1e3) / 1e9
        out[str(N)] = {"shard_rows": rows // N, "ms": round(avg, 4), "frac": round(gbps / HBM_PEAK_GBPS, 4),
                       "kernel_id": plan["kernel_id"], "launches": plan["launches"],
                       "other_launches": plan["other_launches"]}
    return {"emulated": True, "ranks": out,
            "note": "one rank's shard sum at N GPUs, on this GPU; the driver's N-GPU runs measure "
                    "the real thing"}


def separate_alloc_leg(deltas, reps=10):
    """The headline 8-way sum on buffers allocated the way libgeeps allocates
    its oplogs, staging buckets and master versions: one gp_malloc_device per
    buffer (physically contiguous when the device has the range), instead of
    the headline's single arena.  Same bytes, same kernel plan; the bucket
    contents are the headline's deltas copied over.  DESIGN.md §5 (allocation
    spread) has the measured spread over fresh allocations."""
    import ctypes
    from geeps_amd import native
    lib = native.lib()
    stream = torch.cuda.current_stream()
    s = stream.cuda_stream
    n = deltas[0].numel()
    nbytes = n * 4
    ptrs = []
    try:
        for _ in range(len(deltas) + 1):
            p = ctypes.c_void_p()
            native.check(lib.gp_malloc_device(ctypes.byref(p), nbytes), "gp_malloc_device")
            ptrs.append(p.value)
        for p, d in zip(ptrs, deltas):
            native.check(lib.gp_memcpy_async(p, d.data_ptr(), nbytes, s), "gp_memcpy_async")
        master = ptrs[-1]
        native.check(lib.gp_memset_async(master, 0, nbytes, s), "gp_memset_async")
        arr = (ctypes.c_void_p * len(deltas))(*ptrs[:-1])
        fn = lambda: native.check(lib.gp_bucket_sum_apply(master, arr, len(deltas), n, s),
                                  "gp_bucket_sum_apply")
        avg = _time_calls(fn, reps, stream)
    finally:
        torch.cuda.synchronize()
        for p in ptrs:
            lib.gp_free_device(p)
    gbps = (len(deltas) + 2) * nbytes / (avg / 1e3) / 1e9
    return {"ms": round(avg, 4), "GBps": round(gbps, 1), "frac": round(gbps / HBM_PEAK_GBPS, 4),
            "buffers": len(deltas) + 1, "allocator": "gp_malloc_device per buffer (libgeeps' allocation)",
            "note": "the headline sum on separately allocated bucket and master buffers; "
                    "the headline line uses one arena"}


def config2_leg(deltas, master, dev, probe=None, reps=5):
    """BASELINE configs[1]: the same 1M x 1024 shard, 2 client buckets (the
    first two resident deltas, client order 0, 1) summed into the master by one
    gp_bucket_sum_apply.  Algorithmic bytes (2 + 2) * shard bytes."""
    from geeps_amd import rowops
    n = master.numel()
    plan = sum_launch_plan(n, 2)
    stream = torch.cuda.current_stream()
    avg = _time_calls(lambda: rowops.bucket_sum_apply(master, deltas[:2]), reps, stream)
    nbytes = 4 * n * 4
    gbps = nbytes / (avg / 1e3) / 1e9
    rows = n // 1024
    share = plan["share"]  # the dominant kernel's part of the shard
    return {"workload": f"configs[1]: 2 clients, {rows} rows x 1024 fp32, 1 shard, device-resident",
            "ms": round(avg, 4), "GBps": round(gbps, 1), "frac": round(gbps / HBM_PEAK_GBPS, 4),
            "delta_GBps": round(2 * n * 4 / (avg / 1e3) / 1e9, 1), "bytes": nbytes,
            "kernel": plan["kernel"], "launches": plan["launches"],
            "other_launches": plan["other_launches"],
            "avg_launch_ms": round(avg * share / plan["launches"], 5),
            "avg_launch_note": "call time x the dominant kernel's share of the shard / its launches",
            "traffic_source": load_traffic(f"r{rows}_w1024_c2_g1", plan["kernel_id"]),
            "model_ms": (round(model_ms(3 * n * 4, n * 4, probe), 4) if probe else None)}


def main(argv=None, backend="nccl", apply_fn=None):
    """`backend="gloo"` + `apply_fn` exist only for tests/test_bench_dist.py, which
    rehearses this multi-rank flow on CPU ranks; the benchmark itself always
    runs nccl (RCCL) ranks on GPUs with the HIP kernel."""
    args = parse(argv)
    # The libgeeps clock leg runs its worker processes BEFORE this process
    # touches the GPU: this process's own hardware queues would otherwise share
    # the GPU's queue slots with 8 workers and get them time-sliced (the
    # AlexNet-table clock took 50 ms instead of 1.9 ms that way).
    e2e_first = None
    if (backend == "nccl" and int(os.environ.get("WORLD_SIZE", "1")) == 1 and not args.no_e2e
            and torch.cuda.device_count() > 0):
        log("[rank 0] libgeeps end-to-end clock leg (before this process opens the GPU)")
        try:
            e2e_first = libgeeps_leg(args.rows, args.width)
        except Exception as exc:  # a side leg: report it, keep the headline line
            e2e_first = {"error": f"{type(exc).__name__}: {str(exc)[-500:]}"}
    multi_e2e = pre_gpu_multi_leg(args, backend)
    rank, world, dev = init_dist(args.gpus, backend)
    import geeps_amd
    from geeps_amd.shard import ShardedReducer
    geeps_amd.lib()  # the HIP library must be there; no fallback

    R, W, C = args.rows, args.width, args.clients
    from geeps_amd.shard import ShardLayout, hosted_clients
    hosted = hosted_clients(rank, world, C)
    # At N = 1 the buckets are the hosted clients' own buffers: the master shard
    # goes in the same arena, after them.  At N > 1 the timed sum streams the
    # reducer's arena (receive buckets + master), so it is allocated first: a
    # process's first large allocation ran the sum at the top of the spread
    # that later ones land in (allocation spread).
    if world == 1:
        master_floats = ShardLayout(R, W, world, rank).max_rows * W
        deltas, master = make_deltas(hosted, R * W, dev, args.layout, master_floats)
        red = ShardedReducer(R, W, C, dev, exchange=args.exchange, apply_fn=apply_fn,
                             master=master, layout=args.layout)
    else:
        red = ShardedReducer(R, W, C, dev, exchange=args.exchange, apply_fn=apply_fn,
                             layout=args.layout)
        deltas, master = make_deltas(hosted, R * W, dev, args.layout, 0)
    L = red.layout
    log(f"[rank {rank}] shard rows [{L.row_start}, {L.row_start + L.local_rows}) "
        f"hosting clients {red.hosted}, HBM layout {args.layout}")
    red.push(deltas)  # buckets resident on their shard
    _sync(dev)

    wall, kernel_ms = timed_apply(red, args.steps, args.warmup, world, dev)
    wall = max_over_ranks(wall, world, dev)
    avg_kernel_ms = sum(kernel_ms) / len(kernel_ms)
    avg_kernel_ms_max = max_over_ranks(avg_kernel_ms, world, dev)
    plan = sum_launch_plan(L.local_vals, min(C, 8))
    kernel_name, launches = plan["kernel"], plan["launches"]
    step_s = wall / args.steps
    delta_bytes = C * R * W * 4
    value = delta_bytes / step_s / 1e9
    shard_bytes = L.local_vals * 4
    algo_bytes = (C + 2) * shard_bytes           # per step on this rank
    achieved = algo_bytes / (avg_kernel_ms / 1e3) / 1e9
    achieved_min = max_over_ranks(-achieved, world, dev) * -1  # slowest rank

    workload_key = f"r{R}_w{W}_c{C}_g{world}"
    result_exchange = []
    if world > 1 and args.exchange_steps > 0:
        # Both exchanges: "a2a" (RCCL all-to-all, bit-exact client order) and
        # "rs" (RCCL reduce-scatter, ring-order sum), each + N-way sum + all-gather.
        for kind in (args.exchange, "rs" if args.exchange == "a2a" else "a2a"):
            r = red if kind == args.exchange else ShardedReducer(R, W, C, dev, exchange=kind,
                                                                 apply_fn=apply_fn,
                                                                 layout=args.layout)
            log(f"[rank {rank}] {kind} exchange: parity check, then {args.exchange_steps} timed steps")
            chk = exchange_check(r, deltas, R, W, C, dev, world, kind)
            ex = timed_exchange(r, deltas, args.exchange_steps, 1, world, dev)
            ex = max_over_ranks(ex, world, dev) / args.exchange_steps
            result_exchange.append({"ms_per_step": round(ex * 1e3, 3),
                                    "value": round(delta_bytes / ex / 1e9, 2), "unit": "GB/s",
                                    "exchange": kind, "check": chk,
                                    "note": "RCCL bucket exchange + N-way sum + all-gather refresh"})
            if r is not red:
                del r
                if dev.type == "cuda":
                    torch.cuda.empty_cache()

    host_inc = None
    cpu = None
    pmc, pmc_error = None, None
    rowops_res = None
    probe = None
    config2 = None
    e2e = None
    per_rank = None
    sep_alloc = None
    if rank == 0 and world == 1 and dev.type == "cuda":
        if not args.no_hbm_probe:
            log("[rank 0] HBM probes")
            scratch = torch.empty_like(deltas[0])
            probe = hbm_probe(deltas[0], scratch)
            del scratch
        if not args.no_config2 and C >= 2 and master is not None:
            log("[rank 0] configs[1] leg (2 clients)")
            config2 = config2_leg(deltas, master, dev, probe)
        if not args.no_per_rank and master is not None:
            log("[rank 0] per-rank (emulated N-GPU) leg")
            per_rank = per_rank_leg(deltas, master, R, W, dev)
            for v in per_rank["ranks"].values():
                v["predicted_speedup"] = round(avg_kernel_ms / v["ms"], 3)
        if not args.no_separate_alloc and args.layout == "arena":
            log("[rank 0] separate-allocation leg")
            try:
                sep_alloc = separate_alloc_leg(deltas)
            except Exception as exc:  # a side leg (needs another 36 GiB): report, keep the line
                sep_alloc = {"error": f"{type(exc).__name__}: {str(exc)[-300:]}"}
        del deltas
        red = None
        master = None
        torch.cuda.empty_cache()
        if not args.no_rowops:
            log("[rank 0] client row-op leg")
            rowops_res = rowops_leg(R, W, dev, indexes=tuple(args.rowops_index),
                                    only=args.rowops_only, probe=probe)
            torch.cuda.empty_cache()
        e2e = e2e_first
        if not args.no_host_inclusive:
            log("[rank 0] host-inclusive leg")
            host_inc = host_inclusive(R, W, C, dev)
        if not args.no_cpu_baseline:
            log("[rank 0] cpu baseline leg")
            cpu = cpu_baseline(min(args.cpu_rows, R), W, C, args.cpu_seconds)
        # not when this process itself runs under rocprofv3 (it sets ROCPROF_*)
        if not args.no_pmc and not any(k.startswith("ROCPROF") for k in os.environ):
            log("[rank 0] PMC traffic passes (rocprofv3 child processes)")
            pmc, pmc_error = measure_traffic(R, W, C, plan["kernel_id"])

    if rank == 0:
        committed = load_traffic(workload_key, plan["kernel_id"])
        traffic = pmc or committed
        share = plan["share"]
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(step_s * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (uniform [-0.5,0.5) deltas, seed 1000+client)",
            "config": {"workload": f"{C}-way fp32 row reduction into the master table, "
                                   f"{R} rows x {W} fp32, {world} server shard(s), "
                                   f"device-resident (BASELINE.json north-star target: "
                                   f"8-way at 1M x 1024"
                                   + ("; configs[2] shape at 8 shards)" if world > 1 else ")"),
                       "rows": R, "row_width": W, "clients": C, "shards": world,
                       "exchange": args.exchange if world > 1 else "none (resident)",
                       "hbm_layout": args.layout,
                       "parallelism": f"row-range shards x{world}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved_min, 1),
                         "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved_min / HBM_PEAK_GBPS, 4),
                         "traffic": traffic["bytes_per_launch"] if traffic else None,
                         "traffic_source": traffic,
                         "kernel": kernel_name,
                         "kernel_id": plan["kernel_id"],
                         "launches_per_step": launches,
                         "other_launches_per_step": plan["other_launches"],
                         "register_tiles": plan["reg_tiles"],
                         # HIP events around each step's launches on their stream
                         "avg_kernel_ms": round(avg_kernel_ms_max, 4),
                         # per launch of the dominant kernel (its share of the step:
                         # the other launches move the rest of the shard), comparable
                         # with rocprofv3's average for that kernel
                         "avg_launch_ms": round(avg_kernel_ms_max * share / launches, 5),
                         "dominant_share": round(share, 6),
                         "algorithmic_bytes_per_step": algo_bytes,
                         "algorithmic_bytes_per_launch": int(algo_bytes * share / launches)},
            "hbm_GBps_algorithmic": round((C + 2) * R * W * 4 / step_s / 1e9, 1),
            # gradient rows reduced per second (C client rows per table row)
            "rows_per_s": round(C * R / step_s, 1),
            "cpu_baseline": cpu,
        }
        if pmc and committed:
            line["roofline"]["traffic_committed"] = committed
        if pmc_error:
            line["roofline"]["traffic_measure_error"] = pmc_error
        if result_exchange:
            line["exchange_inclusive"] = result_exchange[0]
            line["exchange_inclusive_alt"] = result_exchange[1]
            # configs[2]'s parity on the real ranks, as top-level scalars
            for ex in result_exchange:
                line[f"exchange_ok_{ex['exchange']}"] = ex["check"]["ok"]
                line[f"exchange_max_abs_err_{ex['exchange']}"] = ex["check"]["max_abs_err"]
        if probe:
            line["roofline"]["same_box_copy_GBps"] = probe["copy_GBps"]
            mm = model_ms((C + 1) * shard_bytes, shard_bytes, probe)
            line["roofline"]["same_box_model_ms"] = round(mm, 4)
            line["roofline"]["frac_of_same_box_model"] = round(mm / avg_kernel_ms_max, 4)
            line["hbm_probe"] = probe
        # scalar copies of nested facts: the driver's parsed record keeps a
        # nested object's scalar fields only
        rl = line["roofline"]
        if traffic:
            rl["traffic_over_algorithmic"] = round(traffic["bytes_per_launch"] /
                                                   (algo_bytes * share / launches), 5)
            rl["traffic_measured_in_run"] = bool(pmc)
        if cpu and "all_cores" in cpu:
            cpu["all_cores_GBps"] = round(cpu["all_cores"]["value"], 2)
            cpu["all_cores_threads"] = cpu["all_cores"]["cores"]
            cpu["all_cores_from"] = cpu["all_cores"]["threads_from"]
        if sep_alloc:
            line["roofline"]["separate_alloc"] = sep_alloc
            if "frac" in sep_alloc:
                rl["separate_alloc_frac"] = sep_alloc["frac"]
        if rowops_res:
            for kind in ("random", "identity"):
                for leg in ("scatter_add", "scatter_add_planned", "scatter_init", "scatter_init_planned",
                            "gather", "gather_planned"):
                    v = rowops_res.get(kind, {}).get(leg)
                    if v and "frac" in v:
                        rl[f"rowops_{kind}_{leg}_frac"] = v["frac"]
        if config2:
            rl["config2_frac"] = config2["frac"]
        if e2e:
            for k, v in e2e.items():
                if isinstance(v, dict) and "ms_per_clock" in v:
                    rl[f"libgeeps_{k}_ms_per_clock"] = v["ms_per_clock"]
        if multi_e2e:
            line["libgeeps_multi_gpu"] = multi_e2e
            line.update(multi_gpu_verdict(multi_e2e))
            for k, v in multi_e2e.items():
                if isinstance(v, dict) and "ms_per_clock" in v:
                    rl[f"libgeeps_{k}_ms_per_clock"] = v["ms_per_clock"]
                    rl[f"libgeeps_{k}_read_ok"] = v["read_ok"]
        if config2:
            line["config2"] = config2
        if per_rank:
            line["per_rank_emulation"] = per_rank
        if host_inc:
            line["host_inclusive"] = host_inc
        if rowops_res:
            line["client_rowops"] = rowops_res
        if e2e:
            line["libgeeps_clock"] = e2e
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return line if rank == 0 else None


if __name__ == "__main__":
    main()
