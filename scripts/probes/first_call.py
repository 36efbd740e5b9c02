"""Round-3 probe 6: where the first unplanned call with a new index spends its
time (run under rocprofv3 --kernel-trace --hip-trace --stats).  8 M RowData
rows, random-permutation DoubleIndex: 3 first calls (each with a freshly
allocated index, the plan cache cleared), then 5 steady calls with one index.
Prints the wall time of each call."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from geeps_amd import native, rowops

dev = torch.device("cuda:0")
R, W = 8 << 20, 128
x = torch.rand(R * W, device=dev)
y = torch.zeros(R * W, device=dev)
g = torch.Generator(device="cpu").manual_seed(7)
perm = torch.randperm(R, generator=g)
lib = native.lib()


def call(idx):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rowops.add_rows_from_double_index_gpu(y, x, idx, R)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3


for i in range(3):
    native.check(lib.gp_unplanned_cache_clear(), "cache clear")
    idx = torch.stack([torch.arange(R), perm], 1).to(dev)
    print(f"first call {i}: {call(idx):.3f} ms", flush=True)
for rep in range(2):  # the first pass pays the process's first radix sort (hipCUB load, pool growth)
    native.check(lib.gp_unplanned_cache_clear(), "cache clear")
    idx = torch.stack([torch.arange(R), torch.randperm(R, generator=g)], 1).to(dev)
    for i in range(6):
        print(f"pass {rep} call {i} same index: {call(idx):.3f} ms", flush=True)
