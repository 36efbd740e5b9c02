"""The unplanned calls' steady state on a random index (8 M RowData rows):
after each index's first call, 4 steady scatter-adds, 4 inits and 4 gathers,
for PMC passes (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, one counter a run):
HBM bytes per launch of the inverse-map walk and of the device check against
their algorithmic bytes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from geeps_amd import rowops  # noqa: E402

R, W = 8 << 20, 128
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(5)
x = torch.rand(R * W, generator=g, device=dev)
y = torch.zeros(R * W, device=dev)
idx = torch.stack([torch.arange(R, device=dev), torch.randperm(R, generator=g, device=dev)], 1).contiguous()
for fn in (rowops.add_rows_from_double_index_gpu, rowops.init_rows_from_double_index_gpu):
    for _ in range(5):  # the first call plans; 4 steady calls
        fn(y, x, idx, R, (0, 0), W, R * W, validate=False)
gidx = torch.stack([idx[:, 1], idx[:, 0]], 1).contiguous()
for _ in range(5):
    rowops.assign_rows_to_double_index_gpu(x, y, gidx, R, (0, 0), W, R * W, validate=False)
torch.cuda.synchronize()
print("steady_rowops ok")
