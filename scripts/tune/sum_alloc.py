"""The production N-way sums over fresh allocations (measurement probe, not
product code): is the sweep-form sum's rate a property of the allocation, as
the mixed form's was (alloc_tune)?  Each round allocates the
bench's arena anew (8 buckets + master, 36 GiB, master last) after a spacer of
random size, so the physical pages differ, and times gp_bucket_sum_apply at 8
buckets (the headline), 2 buckets (configs[1]) and the planned init and gather
on an identity index (the no-bucket / zero-input sweeps), 5 calls each (HIP
events, median).

    python scripts/tune/sum_alloc.py [rounds]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from geeps_amd import rowops  # noqa: E402

PEAK = 8000.0


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
    n = 1 << 30  # floats per buffer (4 GiB): the 1M x 1024 table
    R = n // 128
    idx = torch.stack([torch.arange(R, device=dev), torch.arange(R, device=dev)], 1).contiguous()
    splan = rowops.RowPlan(idx, R, (0, 0), 128, R * 128)
    gplan = rowops.RowPlan(idx, R, (0, 0), 128, R * 128, kind="gather")
    del idx
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    print(f"{'round':>5} {'spacer_MiB':>10} {'8-way ms':>9} {'%':>6} {'2-way ms':>9} {'%':>6} "
          f"{'init ms':>8} {'%':>6} {'gather ms':>9} {'%':>6}", flush=True)
    for r in range(rounds):
        spacer_mib = int(torch.randint(1, 4096, (1,), generator=torch.Generator().manual_seed(r)).item())
        spacer = torch.empty(spacer_mib << 18, device=dev)
        arena = torch.empty(9 * n, device=dev)
        torch.rand(8 * n, generator=g, device=dev, out=arena[:8 * n])
        arena[8 * n:].zero_()
        buckets = [arena[k * n:(k + 1) * n] for k in range(8)]
        master = arena[8 * n:]
        t8 = timed(lambda: rowops.bucket_sum_apply(master, buckets))
        t2 = timed(lambda: rowops.bucket_sum_apply(master, buckets[:2]))
        ti = timed(lambda: splan.init(buckets[1], buckets[0]))
        tg = timed(lambda: gplan.gather(buckets[1], buckets[0]))
        f = lambda b, t: b / (t / 1e3) / 1e9 / PEAK * 100  # noqa: E731
        print(f"{r:>5} {spacer_mib:>10} {t8:>9.4f} {f(40 * n, t8):>6.2f} {t2:>9.4f} {f(16 * n, t2):>6.2f} "
              f"{ti:>8.4f} {f(8 * n, ti):>6.2f} {tg:>9.4f} {f(8 * n, tg):>6.2f}", flush=True)
        del spacer, arena, buckets, master
        torch.cuda.empty_cache()
    splan.close()
    gplan.close()


if __name__ == "__main__":
    main()
