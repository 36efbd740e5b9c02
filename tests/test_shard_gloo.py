"""Row-range sharding over 2 (and 4) ranks with the gloo backend on CPU.

Checks, against the oracle applying every client's whole-table delta in client
order 0..N-1 (the reference server's arrival order), that:
  * the a2a exchange + client-order apply + all-gather refresh is bit-exact and
    every rank ends with the identical full table;
  * the reduce-scatter exchange is bit-exact against its own association at 2
    ranks (a two-term sum per shard) and within fp32 tolerance of the client-order
    sum (ring order at 8 ranks);
  * uneven partitions (num_rows % world != 0) use the reference rule
    (clientlib-viter.cpp:674-682) and round-trip through the padded gather.
"""
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from oracle import oracle

import _dist_worker


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _expected(num_rows, W, num_clients, steps):
    m = np.zeros(num_rows * W, np.float32)
    for step in range(steps):
        oracle.apply_updates(m, [oracle.synthetic_delta(c + 100 * step, num_rows * W)
                                 for c in range(num_clients)])
    return m


def _expected_rs_two_ranks(num_rows, W, num_clients, steps):
    m = np.zeros(num_rows * W, np.float32)
    for step in range(steps):
        d = [oracle.synthetic_delta(c + 100 * step, num_rows * W) for c in range(num_clients)]
        oracle.apply_updates(m, [d[2 * j] + d[2 * j + 1] for j in range(num_clients // 2)])
    return m


@pytest.mark.parametrize("world,num_rows,W,clients,exchange,steps", [
    (2, 64, 16, 4, "a2a", 2),
    (2, 37, 12, 2, "a2a", 3),     # uneven rows: 19 + 18
    (4, 41, 8, 8, "a2a", 2),
    (8, 83, 8, 8, "a2a", 2),      # configs[2]'s shape: 8 shards, 8 clients, one per rank
    (8, 83, 8, 8, "rs", 1),
    (2, 64, 16, 4, "rs", 2),
    (2, 37, 12, 2, "rs", 1),
])
def test_sharded_reduction(tmp_path, world, num_rows, W, clients, exchange, steps):
    mp.spawn(_dist_worker.run_shard,
             args=(world, _free_port(), num_rows, W, clients, exchange, steps, str(tmp_path)),
             nprocs=world, join=True)
    e = _expected(num_rows, W, clients, steps)
    tables = [np.load(tmp_path / f"table_{r}.npy") for r in range(world)]
    for r in range(1, world):
        assert np.array_equal(tables[0].view(np.uint32), tables[r].view(np.uint32))
    hosted = sorted(int(c) for r in range(world) for c in np.load(tmp_path / f"hosted_{r}.npy"))
    assert hosted == list(range(clients))
    if exchange == "a2a":
        assert np.array_equal(tables[0].view(np.uint32), e.view(np.uint32))
    elif world == 2:
        # two ranks: each shard's reduce-scatter adds exactly two deltas, and a
        # two-term fp32 sum is the same in either order, so the rs form is
        # pinned bit for bit: master += (d[2j] + d[2j+1]) for hosted slot j
        assert np.array_equal(tables[0].view(np.uint32), _expected_rs_two_ranks(num_rows, W, clients, steps)
                              .view(np.uint32))
        np.testing.assert_allclose(tables[0], e, rtol=0,
                                   atol=clients * steps * np.finfo(np.float32).eps * (0.5 * clients * steps + 1))
    else:
        # per element: |err| <= (N*steps) ulps of the largest partial sum
        tol = clients * steps * np.finfo(np.float32).eps * (0.5 * clients * steps + 1)
        np.testing.assert_allclose(tables[0], e, rtol=0, atol=tol)


def test_world_one_is_local():
    import torch
    from geeps_amd.shard import ShardedReducer
    red = ShardedReducer(10, 4, 3, device="cpu", apply_fn=_dist_worker.oracle_apply)
    assert red.hosted == [0, 1, 2]
    deltas = [torch.from_numpy(oracle.synthetic_delta(c, 40)) for c in range(3)]
    t = red.step(deltas)
    assert np.array_equal(t.numpy().view(np.uint32), _expected(10, 4, 3, 1).view(np.uint32))


def test_hosting_requires_divisible_clients():
    from geeps_amd.shard import hosted_clients
    assert hosted_clients(1, 4, 8) == [1, 5]
    with pytest.raises(ValueError):
        hosted_clients(0, 3, 8)
