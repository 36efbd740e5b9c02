"""Row-op legs over fresh allocations (tuning probe, not product code): is the
identity-index scatter-add / init time a property of the allocation, as the
mixed-form bucket sum's was (alloc_tune)?  Each round allocates
x and y anew (with a spacer of random size before them, so the physical pages
differ), then times the planned add, the planned init and the gather on an
identity and a random index, 5 calls each (HIP events).

    python scripts/tune/rowop_alloc.py [rounds]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from geeps_amd import rowops  # noqa: E402


def timed(fn, reps=5):
    fn()
    s = torch.cuda.current_stream()
    out = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        fn()
        b.record(s)
        b.synchronize()
        out.append(a.elapsed_time(b))
    return sorted(out)[len(out) // 2]


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    dev = torch.device("cuda:0")
    R = 1 << 23
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    idx_id = torch.stack([torch.arange(R, device=dev), torch.arange(R, device=dev)], 1).contiguous()
    idx_rnd = torch.stack([torch.arange(R, device=dev), torch.randperm(R, generator=g, device=dev)],
                          1).contiguous()
    plans = {"identity": rowops.RowPlan(idx_id, R, (0, 0), 128, R * 128),
             "random": rowops.RowPlan(idx_rnd, R, (0, 0), 128, R * 128)}
    add_b, init_b = 3 * R * 512 + 16 * R, 2 * R * 512 + 16 * R
    print(f"{'round':>5} {'spacer_MiB':>10} " + " ".join(f"{k:>22}" for k in
          ("id add", "id init", "id gather", "rnd add", "rnd init", "rnd gather", "dense add",
           "D2D copy")), flush=True)
    for r in range(rounds):
        spacer_mib = int(torch.randint(1, 4096, (1,)).item())
        spacer = torch.empty(spacer_mib << 18, device=dev)
        x = torch.rand(R * 128, generator=g, device=dev)
        y = torch.rand(R * 128, generator=g, device=dev)
        cols = []
        for kind, idx in (("identity", idx_id), ("random", idx_rnd)):
            p = plans[kind]
            for name, fn, nb in (("add", lambda: p.add(y, x), add_b),
                                 ("init", lambda: p.init(y, x), init_b),
                                 ("gather", lambda: rowops.assign_rows_to_double_index_gpu(
                                     x, y, idx, R, (0, 0), 128, R * 128, validate=False), init_b)):
                ms = timed(fn)
                cols.append(f"{ms:8.4f} ms {nb / ms / 1e9 / 8:6.1%}")
        # the dense forms over the same buffers: gp_add (y = y + x, the phased
        # 1-bucket sum) and a hipMemcpyAsync copy (1 read + 1 write stream)
        ms = timed(lambda: rowops.gpu_add(R * 128, y, x, y))
        cols.append(f"{ms:8.4f} ms {3 * R * 512 / ms / 1e9 / 8:6.1%}")
        ms = timed(lambda: y.copy_(x))
        cols.append(f"{ms:8.4f} ms {2 * R * 512 / ms / 1e9 / 8:6.1%}")
        print(f"{r:>5} {spacer_mib:>10} " + " ".join(f"{c:>22}" for c in cols), flush=True)
        del x, y, spacer
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
