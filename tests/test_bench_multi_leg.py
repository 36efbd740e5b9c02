"""bench.py --gpus N's drop-in leg, control flow only (CPU): rank 0 runs the
one-process-per-GPU libgeeps leg while every other rank waits on a file store
without touching a GPU, then all ranks go on.
The leg itself is stubbed here (it needs N GPUs); a leg that raises still
releases the other ranks and is reported, not fatal."""
import multiprocessing as mp
import os
import socket
import sys
import time
from types import SimpleNamespace

import pytest

from conftest import REPO


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, fail, out):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_PORT=str(port))
    sys.path.insert(0, REPO)
    import bench

    def leg(n, rows, W):
        time.sleep(1.0)  # the other ranks must still be waiting
        if fail:
            raise RuntimeError("stub leg failed")
        return {"processes": n, "rows": rows, "W": W, "done_at": time.time()}

    bench.libgeeps_multi_gpu_leg = leg
    args = SimpleNamespace(no_e2e=False, no_multi_e2e=False, rows=1024, width=8)
    res = bench.pre_gpu_multi_leg(args, "nccl")
    out.put((rank, res, time.time()))


@pytest.mark.parametrize("world,fail", [(2, False), (4, False), (2, True)])
def test_rank0_runs_the_leg_while_the_others_wait(world, fail):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, fail, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        rank, res, t = q.get(timeout=120)
        got[rank] = (res, t)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res0, _ = got[0]
    if fail:
        assert "stub leg failed" in res0["error"]
    else:
        assert res0["processes"] == world and res0["rows"] == 1024 and res0["W"] == 8
        for r in range(1, world):
            assert got[r][0] is None
            assert got[r][1] >= res0["done_at"]  # released only after the leg finished


def test_world_one_and_other_backends_skip_the_leg():
    sys.path.insert(0, REPO)
    import bench
    args = SimpleNamespace(no_e2e=False, no_multi_e2e=False, rows=1024, width=8)
    assert bench.pre_gpu_multi_leg(args, "nccl") is None  # WORLD_SIZE unset: N = 1
    os.environ["WORLD_SIZE"] = "2"
    try:
        assert bench.pre_gpu_multi_leg(args, "gloo") is None
        assert bench.pre_gpu_multi_leg(SimpleNamespace(no_e2e=False, no_multi_e2e=True, rows=1, width=1),
                                       "nccl") is None
    finally:
        del os.environ["WORLD_SIZE"]


class _FakeClockBench:
    """Stands in for scripts/run_clock_bench.py: records the runs, sleeps `cost` s each."""
    BIN = __file__

    def __init__(self, cost=0.0, fail_on=None):
        self.calls, self.cost, self.fail_on = [], cost, fail_on

    def run(self, P, rows, clocks, warmup, slack, transport, timeout, extra_env):
        path = "staged" if extra_env["GEEPS_STAGE_PEER_UPDATES"] == "1" else "in_place"
        self.calls.append((rows, path, timeout))
        time.sleep(self.cost)
        if self.fail_on == (len(self.calls) - 1):
            raise RuntimeError("fake failure")
        return {"ms_per_clock_max": 1.0, "aggregate_delta_GBps": 1.0, "read_ok": True, "read_checked": 1,
                "devices": list(range(P))}


def _leg(monkeypatch, fake, budget=None):
    sys.path.insert(0, REPO)
    import bench
    monkeypatch.setattr(bench, "_clock_bench_module", lambda: fake)
    if budget is not None:
        monkeypatch.setenv("GEEPS_BENCH_MULTI_BUDGET_S", str(budget))
    return bench.libgeeps_multi_gpu_leg(8, 1024, 1024, gpus_seen=8)


def test_leg_runs_the_staged_path_first_within_its_budget(monkeypatch):
    fake = _FakeClockBench()
    out = _leg(monkeypatch, fake)
    assert [c[1] for c in fake.calls] == ["staged", "staged", "in_place", "in_place"]
    assert all(out[k]["read_ok"] for k in ("1Mx1024_staged", "alexnet_staged", "1Mx1024_in_place",
                                           "alexnet_in_place"))
    assert all(c[2] <= 150 for c in fake.calls)
    # a spent budget skips the rest (the scaling runs after it stay short)
    fake = _FakeClockBench(cost=0.3)
    out = _leg(monkeypatch, fake, budget=20.5)
    assert len(fake.calls) == 2 and "budget" in out["alexnet_in_place"]["skipped"]


def test_leg_stops_at_its_first_failure(monkeypatch):
    fake = _FakeClockBench(fail_on=0)
    out = _leg(monkeypatch, fake)
    assert len(fake.calls) == 1 and "fake failure" in out["1Mx1024_staged"]["error"]
    assert all("after 1Mx1024_staged failed" in out[k]["skipped"]
               for k in ("alexnet_staged", "1Mx1024_in_place", "alexnet_in_place"))


def test_multi_gpu_verdict_settles_the_default_from_one_record():
    """the leg's record alone says whether libgeeps'
    cross-GPU default (staged) is no slower than in place, per table and
    overall, as top-level scalars."""
    sys.path.insert(0, REPO)
    import bench

    def rec(ms, ok=True):
        return {"ms_per_clock": ms, "read_ok": ok}
    multi = {"1Mx1024_staged": rec(19.0), "1Mx1024_in_place": rec(25.0),
             "alexnet_staged": rec(2.0), "alexnet_in_place": rec(1.96)}  # within the 3 % band
    v = bench.multi_gpu_verdict(multi)
    assert v["libgeeps_multi_gpu_default_path"] == "staged"
    assert v["libgeeps_multi_gpu_1Mx1024_staged_ms_per_clock"] == 19.0
    assert v["libgeeps_multi_gpu_1Mx1024_in_place_ms_per_clock"] == 25.0
    assert v["libgeeps_multi_gpu_1Mx1024_faster_path"] == "staged"
    assert v["libgeeps_multi_gpu_alexnet_faster_path"] == "in_place"
    assert v["libgeeps_multi_gpu_alexnet_default_ok"] is True
    assert v["libgeeps_multi_gpu_default_ok"] is True
    assert all(not isinstance(x, (dict, list)) for x in v.values())  # scalars only
    multi["1Mx1024_staged"] = rec(30.0)
    v = bench.multi_gpu_verdict(multi)
    assert v["libgeeps_multi_gpu_1Mx1024_default_ok"] is False and v["libgeeps_multi_gpu_default_ok"] is False
    # a path not measured (skipped, failed, a Read not exact): not decided
    for broken in ({"skipped": "budget"}, {"error": "x"}, rec(1.0, ok=False)):
        m = dict(multi, alexnet_in_place=broken)
        v = bench.multi_gpu_verdict(m)
        assert v["libgeeps_multi_gpu_alexnet_default_ok"] is None and v["libgeeps_multi_gpu_default_ok"] is None
