"""CPU rehearsal of bench.py's multi-rank flow (the driver runs the real thing
on 1/2/4/8 MI355X with RCCL): gloo ranks on CPU, the oracle standing in for the
HIP apply kernel.  Checks the JSON contract fields and that the exchange leg and
max-over-ranks timing run at world sizes 2 and 4."""
import json
import socket

import pytest
import torch.multiprocessing as mp

import _dist_worker


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,exchange", [(2, "a2a"), (4, "a2a"), (2, "rs"), (8, "a2a")])
def test_bench_multirank_flow(tmp_path, world, exchange):
    argv = ["--gpus", str(world), "--steps", "2", "--warmup", "1", "--rows", "1000", "--width", "64",
            "--clients", "8", "--exchange", exchange, "--exchange-steps", "2"]
    mp.spawn(_dist_worker.run_bench, args=(world, _free_port(), argv, str(tmp_path)), nprocs=world,
             join=True)
    line = json.load(open(tmp_path / "bench.json"))
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in line, k
    assert line["n_gpus"] == world and line["steps"] == 2 and line["scaling"] == "strong"
    assert line["value"] > 0 and line["roofline"]["bound"] == "hbm"
    assert line["config"]["shards"] == world and line["config"]["exchange"] == exchange
    assert line["exchange_inclusive"]["value"] > 0
    assert line["exchange_inclusive"]["exchange"] == exchange
    assert line["exchange_inclusive_alt"]["exchange"] != exchange
    assert line["cpu_baseline"] is None  # rank-0 CPU baseline runs only at N = 1
