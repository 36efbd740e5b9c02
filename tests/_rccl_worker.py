"""One rank of tests/test_rccl.py's configs[2] check (launched by
torch.distributed.run, one process per GPU, RCCL = backend "nccl").

For each table size and each exchange ("a2a": RCCL all-to-all, the N-way sum
in client order; "rs": RCCL reduce-scatter), one clean clock of
geeps_amd.shard.ShardedReducer on a zeroed master -- push -> the HIP N-way
sum -> all-gather -- checked on every rank by bench.exchange_check (every
element against the client-order sum of the regenerated deltas, sampled rows
against a numpy restatement), and on rank 0 for the reduced table every
element against the oracle's apply_updates in client order
(src/server/tablet-server.cpp:119-134).  Writes rank 0's results as JSON.

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P tests/_rccl_worker.py OUT.json ROWSxW[,ROWSxW...]
"""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main(out_path, sizes):
    local = int(os.environ["LOCAL_RANK"])
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", local)
    import bench
    import geeps_amd
    from geeps_amd.shard import ShardedReducer, hosted_clients
    geeps_amd.lib()  # the HIP library must load: no fallback
    C = 8
    results = []
    try:
        for R, W in sizes:
            hosted = hosted_clients(rank, world, C)
            deltas, _ = bench.make_deltas(hosted, R * W, dev, "separate")
            for kind in ("a2a", "rs"):
                red = ShardedReducer(R, W, C, dev, exchange=kind)
                chk = bench.exchange_check(red, deltas, R, W, C, dev, world, kind)
                oracle_ok = None
                if R * W <= (1 << 23):  # reduced table: every element against the oracle on rank 0
                    table = red.refreshed[:R * W].cpu().numpy()
                    if rank == 0:
                        from oracle import oracle
                        m = np.zeros(R * W, np.float32)
                        oracle.apply_updates(m, [bench.regen_delta(c, R * W, dev).cpu().numpy()
                                                 for c in range(C)])
                        if kind == "a2a":
                            oracle_ok = bool(np.array_equal(table.view(np.uint32), m.view(np.uint32)))
                        else:
                            oracle_ok = bool(np.abs(table - m).max() <= bench.rs_tolerance(C))
                results.append({"rows": R, "width": W, "exchange": kind, "check": chk,
                                "oracle_ok": oracle_ok, "world": world})
                del red
                torch.cuda.empty_cache()
            del deltas
            torch.cuda.empty_cache()
        if rank == 0:
            with open(out_path, "w") as f:
                json.dump(results, f)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    sizes = [tuple(int(x) for x in s.split("x")) for s in sys.argv[2].split(",")]
    main(sys.argv[1], sizes)
