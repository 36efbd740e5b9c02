"""Worker bodies for the multi-process (gloo, CPU) tests of geeps_amd.shard.

The exchange / partition / refresh logic runs exactly as on the GPU; only the
apply step is swapped for the CPU oracle (the HIP kernel needs a device), which
is test infrastructure standing in for the kernel under test elsewhere.
"""
import os

import numpy as np
import torch
import torch.distributed as dist


def oracle_apply(master: torch.Tensor, buckets) -> None:
    from oracle import oracle
    m = master.numpy()
    oracle.apply_updates(m, [b.contiguous().numpy() for b in buckets])


def hip_apply(master: torch.Tensor, buckets) -> None:
    """The HIP N-way sum on cuda:0 for a CPU-resident rank (the gloo-exchange
    rehearsal of tests/test_rccl.py on a one-GPU box): master and buckets go to
    the device, gp_bucket_sum_apply sums them in client order, master comes back."""
    from geeps_amd.rowops import bucket_sum_apply
    dev = torch.device("cuda", 0)
    m = master.to(dev)
    bucket_sum_apply(m, [b.contiguous().to(dev) for b in buckets])
    torch.cuda.synchronize()
    master.copy_(m.cpu())


def full_delta(c: int, num_rows: int, W: int) -> torch.Tensor:
    from oracle import oracle
    return torch.from_numpy(oracle.synthetic_delta(c, num_rows * W))


def run_shard(rank, world, port, num_rows, W, num_clients, exchange, steps, out_dir, apply="oracle"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from geeps_amd.shard import ShardedReducer
        red = ShardedReducer(num_rows, W, num_clients, device="cpu", exchange=exchange,
                             apply_fn=oracle_apply if apply == "oracle" else hip_apply)
        for step in range(steps):
            deltas = [full_delta(c + 100 * step, num_rows, W) for c in red.hosted]
            table = red.step(deltas)
        np.save(os.path.join(out_dir, f"table_{rank}.npy"), table.numpy()[:num_rows * W])
        np.save(os.path.join(out_dir, f"hosted_{rank}.npy"), np.array(red.hosted))
    finally:
        dist.destroy_process_group()


def run_rehearsal(rank, world, port, num_rows, W, num_clients, exchange, steps, out_dir, apply="hip"):
    """configs[2]'s flow at its own rank count on one box (tests/test_rccl.py):
    `steps` clocks of ShardedReducer.step over gloo ranks with the oracle's
    seeded deltas, then bench.exchange_check -- the check `bench.py --gpus N`
    runs on its RCCL ranks -- on the same reducer.  Rank 0 saves its refreshed
    table; every rank writes a digest of its own and the check's result."""
    import hashlib
    import json
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from geeps_amd.shard import ShardedReducer
        red = ShardedReducer(num_rows, W, num_clients, device="cpu", exchange=exchange,
                             apply_fn=oracle_apply if apply == "oracle" else hip_apply)
        for step in range(steps):
            deltas = [full_delta(c + 100 * step, num_rows, W) for c in red.hosted]
            table = red.step(deltas)
            del deltas
            if exchange == "rs":  # the buckets gloo's reduce-scatter delivered to this shard, per slot
                for j, r in enumerate(red.recv):
                    np.save(os.path.join(out_dir, f"rs_{rank}_{step}_{j}.npy"), r[:red.layout.local_vals].numpy())
        table = table.numpy()[:num_rows * W]
        if rank == 0:
            np.save(os.path.join(out_dir, "table_0.npy"), table)
        digest = hashlib.sha256(table.tobytes()).hexdigest()
        del table
        cpu = torch.device("cpu")
        bdeltas, _ = bench.make_deltas(red.hosted, num_rows * W, cpu, "separate")
        chk = bench.exchange_check(red, bdeltas, num_rows, W, num_clients, cpu, world, exchange)
        with open(os.path.join(out_dir, f"rank_{rank}.json"), "w") as f:
            json.dump({"rank": rank, "hosted": red.hosted, "digest": digest, "check": chk,
                       "shard": [red.layout.row_start, red.layout.local_rows]}, f)
    finally:
        dist.destroy_process_group()


def run_bench(rank, world, port, argv, out_dir):
    """bench.py's multi-rank flow on gloo CPU ranks (oracle as the apply step)."""
    import json
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world)})
    import bench
    line = bench.main(argv, backend="gloo", apply_fn=oracle_apply)
    if rank == 0:
        with open(os.path.join(out_dir, "bench.json"), "w") as f:
            json.dump(line, f)


def run_bad_split_check(rank, world, port, out_dir):
    """bench.exchange_check on a reducer whose exchange reads every client's
    slices one row off (what a wrong all-to-all split offset would do): the
    check must fail on every rank."""
    import json
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from geeps_amd.shard import ShardedReducer

        R, W, C = 37, 8, 4

        class OffByOneRow(ShardedReducer):
            def push(self, deltas):
                super().push([torch.roll(d, W) for d in deltas])

        red = OffByOneRow(R, W, C, device="cpu", exchange="a2a", apply_fn=oracle_apply)
        deltas, _ = bench.make_deltas(red.hosted, R * W, torch.device("cpu"), "separate")
        res = bench.exchange_check(red, deltas, R, W, C, torch.device("cpu"), world, "a2a")
        if rank == 0:
            with open(os.path.join(out_dir, "check.json"), "w") as f:
                json.dump(res, f)
    finally:
        dist.destroy_process_group()
