"""Where the first unplanned call with a new index spends its time (8 M
RowData rows, random permutation of destinations): three fresh index tensors,
each called twice (plan + first steady call), host wall time per call and HIP
event time on the stream.  Run under rocprofv3 --kernel-trace --stats for the
per-kernel split."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from geeps_amd import native, rowops  # noqa: E402

R, W = 8 << 20, 128
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(5)
x = torch.rand(R * W, generator=g, device=dev)
y = torch.zeros(R * W, device=dev)
stream = torch.cuda.current_stream()
out = []
for op in ("add", "init"):
    fn = rowops.add_rows_from_double_index_gpu if op == "add" else rowops.init_rows_from_double_index_gpu
    for trial in range(3):
        idx = torch.stack([torch.arange(R, device=dev), torch.randperm(R, generator=g, device=dev)], 1).contiguous()
        torch.cuda.synchronize()
        for call in range(2):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            a.record(stream)
            fn(y, x, idx, R, (0, 0), W, R * W, validate=False)
            b.record(stream)
            t1 = time.perf_counter()
            b.synchronize()
            out.append({"op": op, "trial": trial, "call": call, "host_ms": round((t1 - t0) * 1e3, 3),
                        "gpu_ms": round(a.elapsed_time(b), 4)})
        del idx
    native.check(native.lib().gp_unplanned_cache_clear(), "gp_unplanned_cache_clear")
print(json.dumps(out))
