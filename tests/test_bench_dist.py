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


@pytest.mark.parametrize("world,exchange,rows", [(2, "a2a", 1000), (4, "a2a", 1000), (2, "rs", 1000),
                                                (8, "a2a", 1000), (8, "rs", 1003), (4, "a2a", 1001)])
def test_bench_multirank_flow(tmp_path, world, exchange, rows):
    argv = ["--gpus", str(world), "--steps", "2", "--warmup", "1", "--rows", str(rows), "--width", "64",
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
    # configs[2]'s parity check ran on every rank for both exchanges
    # (uneven partitions: 1003 rows over 8, 1001 over 4)
    for kind in ("a2a", "rs"):
        assert line[f"exchange_ok_{kind}"] is True, line
        chk = line["exchange_inclusive" if kind == exchange else "exchange_inclusive_alt"]["check"]
        assert chk["ok"] and chk["elements_checked"] == rows * 64 and chk["ranks"] == world
        assert chk["rows_sampled"] >= 2 * world
    assert line["exchange_max_abs_err_a2a"] == 0.0
    assert 0.0 <= line["exchange_max_abs_err_rs"] <= 8 * 1.2e-7 * 5


def test_exchange_check_catches_a_wrong_split(tmp_path):
    """The check is not vacuous: a reducer whose all-to-all split is off by one
    row (a wrong shard offset on the real ranks) fails it on gloo."""
    mp.spawn(_dist_worker.run_bad_split_check, args=(2, _free_port(), str(tmp_path)), nprocs=2,
             join=True)
    res = json.load(open(tmp_path / "check.json"))
    assert res["ok"] is False and res["max_abs_err"] > 0
