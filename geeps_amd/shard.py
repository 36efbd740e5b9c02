"""Row-range sharding of the parameter table over ranks (one rank per GPU).

The reference shards each table by contiguous row range over tablet servers
(``per_server_row_start[i] = div*i + min(i, res)``,
src/client/clientlib-viter.cpp:674-682).  A clock's exchange is hand-rolled over
ZeroMQ: every client sends each server its row slice (functionally a
reduce-scatter, the reduction done at the server: src/client/clientlib-data.cpp:487-509),
each server sums the slices into its master copy (src/server/tablet-server.cpp:119-134)
and replies its whole shard to every client (functionally an all-gather,
src/server/tablet-server.cpp:136-163).

Here the same three steps run over RCCL (``torch.distributed`` backend "nccl"
= RCCL on ROCm, over xGMI inside a node), with the reduction on the device:

  1. exchange  — "a2a" (default, deterministic): one all-to-all per hosted
     client slot moves every client's slice for shard s to rank s unreduced;
     "rs": RCCL reduce-scatter sums the slices in flight (ring order, not
     client order: held to a tolerance, not bit-exact).
  2. apply     — ``gp_bucket_sum_apply`` adds all N buckets to the master shard
     in client-id order 0..N-1 (bit-identical to the reference applying the N
     messages in that arrival order).
  3. refresh   — all-gather of the (padded) master shards.

Clients are synthetic and hosted round-robin: client ``c`` lives on rank
``c % world``; every rank hosts ``num_clients // world`` of them.

``apply_fn`` exists so the gloo/CPU tests can exercise the exchange and
partition logic with the oracle standing in for the HIP kernel; the product
default is the HIP kernel and nothing here falls back to the CPU.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Sequence

import torch
import torch.distributed as dist


def server_partition(num_rows: int, num_servers: int):
    """(row_start, num_rows) per server — clientlib-viter.cpp:674-682."""
    if num_servers <= 0:
        raise ValueError("num_servers must be positive")
    div, res = divmod(num_rows, num_servers)
    starts = [div * i + min(i, res) for i in range(num_servers)]
    counts = [div + (1 if i < res else 0) for i in range(num_servers)]
    return starts, counts


def hosted_clients(rank: int, world: int, num_clients: int) -> list[int]:
    if num_clients % world:
        raise ValueError("num_clients must be a multiple of the world size")
    return [c for c in range(num_clients) if c % world == rank]


def _default_apply(master: torch.Tensor, buckets: Sequence[torch.Tensor]) -> None:
    from .rowops import bucket_sum_apply
    bucket_sum_apply(master, buckets)


@dataclass
class ShardLayout:
    num_rows: int
    row_size: int
    world: int
    rank: int

    def __post_init__(self):
        self.starts, self.counts = server_partition(self.num_rows, self.world)
        self.max_rows = max(self.counts)

    @property
    def row_start(self) -> int:
        return self.starts[self.rank]

    @property
    def local_rows(self) -> int:
        return self.counts[self.rank]

    @property
    def local_vals(self) -> int:
        return self.local_rows * self.row_size


class ShardedReducer:
    """One rank's server shard plus its hosted synthetic clients.

    ``deltas[j]`` is the full-table delta buffer (num_rows * row_size floats) of
    hosted client ``hosted[j]``.  ``push()`` runs the exchange, ``apply()`` the
    device-resident N-way sum, ``refresh()`` the all-gather.
    """

    def __init__(self, num_rows: int, row_size: int, num_clients: int, device,
                 group=None, exchange: str = "a2a",
                 apply_fn: Callable | None = None, master: torch.Tensor | None = None,
                 layout: str = "arena"):
        if exchange not in ("a2a", "rs"):
            raise ValueError("exchange must be 'a2a' or 'rs'")
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.layout = ShardLayout(num_rows, row_size, self.world, self.rank)
        self.num_clients = num_clients
        self.hosted = hosted_clients(self.rank, self.world, num_clients)
        self.exchange = exchange
        self.device = device
        self.apply_fn = apply_fn or _default_apply
        if layout not in ("arena", "separate"):
            raise ValueError("layout must be 'arena' or 'separate'")
        L = self.layout
        self.hbm_layout = layout
        self.refreshed = None
        self.recv: list[torch.Tensor] = []
        self._buckets: list[torch.Tensor] = []
        # HBM layout of the shard: with "arena" the exchange's receive buckets
        # and the master shard (padded to max_rows so the all-gather counts are
        # equal) are carved from ONE allocation, master last — the placement
        # that measured fastest for the N-way sum (profiles/r01/bucket_tune_sweep6_layout.txt).
        padded = L.max_rows * row_size
        if master is not None:
            if master.numel() < padded:
                raise ValueError("master too small for the shard")
            self.master = master[:padded]
            self.master.zero_()
        elif layout == "arena" and self.world > 1:
            per = (self.world * L.local_vals) if exchange == "a2a" else padded
            arena = torch.empty(len(self.hosted) * per + padded, dtype=torch.float32,
                                device=device)
            self.recv = [arena[j * per:(j + 1) * per] for j in range(len(self.hosted))]
            self.master = arena[len(self.hosted) * per:]
            self.master.zero_()
        else:
            self.master = torch.zeros(padded, dtype=torch.float32, device=device)

    # -- exchange -----------------------------------------------------------
    def push(self, deltas: Sequence[torch.Tensor]) -> None:
        """Move the hosted clients' row slices to their owning shards."""
        L = self.layout
        if len(deltas) != len(self.hosted):
            raise ValueError("one delta buffer per hosted client")
        for d in deltas:
            if d.numel() != L.num_rows * L.row_size:
                raise ValueError("delta buffer must cover the whole table")
        if self.world == 1:
            self._buckets = list(deltas)  # already resident: client order == hosted order
            return
        W = L.row_size
        split_in = [c * W for c in L.counts]
        if self.exchange == "a2a":
            if not self.recv:
                self.recv = [torch.empty(self.world * L.local_vals, dtype=torch.float32,
                                         device=self.device) for _ in self.hosted]
            for j, d in enumerate(deltas):
                dist.all_to_all_single(self.recv[j], d, [L.local_vals] * self.world, split_in,
                                       group=self.group)
            # slot j, source rank r carries client j*world + r: client-id order
            n = L.local_vals
            self._buckets = [self.recv[j][r * n:(r + 1) * n]
                             for j in range(len(self.hosted)) for r in range(self.world)]
        else:
            # reduce-scatter needs equal counts: pad each delta to max_rows per shard
            padded = L.max_rows * W
            if not self.recv:
                self.recv = [torch.empty(padded, dtype=torch.float32, device=self.device)
                             for _ in self.hosted]
            if not hasattr(self, "_send"):
                self._send = torch.zeros(self.world * padded, dtype=torch.float32,
                                         device=self.device)
            for j, d in enumerate(deltas):
                if all(c == L.max_rows for c in L.counts):
                    src = d
                else:
                    for s in range(self.world):
                        a, c = L.starts[s] * W, L.counts[s] * W
                        self._send[s * padded:s * padded + c].copy_(d[a:a + c])
                    src = self._send
                dist.reduce_scatter_tensor(self.recv[j], src, group=self.group)
            self._buckets = [r[:L.local_vals] for r in self.recv]

    # -- device-resident reduction -----------------------------------------
    def apply(self) -> None:
        """master_shard += buckets, in client order (one device pass)."""
        if not self._buckets:
            return
        L = self.layout
        if self.world == 1:
            buckets = self._buckets
        else:
            buckets = [b[:L.local_vals] for b in self._buckets]
        self.apply_fn(self.master[:L.local_vals], buckets)

    # -- refresh ------------------------------------------------------------
    def refresh(self) -> torch.Tensor:
        """All-gather the master shards; returns the full table (num_rows*W)."""
        L = self.layout
        if self.world == 1:
            self.refreshed = self.master
            return self.master
        if self.refreshed is None:
            self._gathered = torch.empty(self.world * L.max_rows * L.row_size,
                                         dtype=torch.float32, device=self.device)
        dist.all_gather_into_tensor(self._gathered, self.master, group=self.group)
        if all(c == L.max_rows for c in L.counts):
            self.refreshed = self._gathered
        else:
            if self.refreshed is None or self.refreshed is self._gathered:
                self.refreshed = torch.empty(L.num_rows * L.row_size, dtype=torch.float32,
                                             device=self.device)
            W, P = L.row_size, L.max_rows * L.row_size
            for s in range(self.world):
                self.refreshed[L.starts[s] * W:(L.starts[s] + L.counts[s]) * W].copy_(
                    self._gathered[s * P:s * P + L.counts[s] * W])
        return self.refreshed

    def step(self, deltas: Sequence[torch.Tensor]) -> torch.Tensor:
        """One clock: exchange, apply, refresh."""
        self.push(deltas)
        self.apply()
        return self.refresh()
