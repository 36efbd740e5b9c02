"""ctypes wrapper of oracle/oracle.c — the CPU restatement of the reference path.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by geeps_amd/.  See oracle.c for the parity
status ("parity unpinned" for the arithmetic; layout pinned against the
reference headers).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")

_lib = None
_fp = ctypes.POINTER(ctypes.c_float)
_u64p = ctypes.POINTER(ctypes.c_uint64)


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE, "build/liboracle.so"], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        rowop = [_fp, _fp, _u64p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint64,
                 ctypes.c_size_t, ctypes.c_size_t]
        for name in ("oracle_add_rows_from_double_index", "oracle_assign_rows_to_double_index",
                     "oracle_assign_rows_from_double_index"):
            getattr(L, name).argtypes = rowop
            getattr(L, name).restype = None
        L.oracle_vs_add.argtypes = [ctypes.c_int64, _fp, _fp, _fp]
        L.oracle_vs_add.restype = ctypes.c_int
        L.oracle_apply_updates.argtypes = [_fp, ctypes.POINTER(_fp), ctypes.c_int, ctypes.c_int64]
        L.oracle_apply_updates.restype = ctypes.c_int
        L.oracle_apply_updates_mt.argtypes = [_fp, ctypes.POINTER(_fp), ctypes.c_int,
                                              ctypes.c_int64, ctypes.c_int]
        L.oracle_apply_updates_mt.restype = ctypes.c_int
        L.oracle_server_partition.argtypes = [ctypes.c_size_t, ctypes.c_size_t, _u64p, _u64p]
        L.oracle_server_partition.restype = None
        L.oracle_fill_uniform.argtypes = [_fp, ctypes.c_int64, ctypes.c_uint64, ctypes.c_int]
        L.oracle_fill_uniform.restype = ctypes.c_int
        _lib = L
    return _lib


def _f(a: np.ndarray):
    assert a.dtype == np.float32 and a.flags.c_contiguous
    return a.ctypes.data_as(_fp)


def _idx(index: np.ndarray):
    index = np.ascontiguousarray(index, dtype=np.uint64).reshape(-1, 2)
    return index, index.ctypes.data_as(_u64p)


_NO_LIMIT = (1 << 64) - 1


def _rowop(name, y, x, index, offset, row_size, num_vals_limit):
    index, ip = _idx(index)
    limit = _NO_LIMIT if num_vals_limit is None else int(num_vals_limit)
    getattr(lib(), name)(_f(y), _f(x), ip, index.shape[0], int(offset[0]), int(offset[1]),
                         int(row_size), limit)


def add_rows_from_double_index(y, x, index, offset=(0, 0), row_size=128, num_vals_limit=None):
    """In place on ``y``; reference src/common/row-op-util.hpp:121-139."""
    _rowop("oracle_add_rows_from_double_index", y, x, index, offset, row_size, num_vals_limit)


def assign_rows_to_double_index(y, x, index, offset=(0, 0), row_size=128, num_vals_limit=None):
    """In place on ``y``; reference src/common/row-op-util.hpp:81-99."""
    _rowop("oracle_assign_rows_to_double_index", y, x, index, offset, row_size, num_vals_limit)


def assign_rows_from_double_index(y, x, index, offset=(0, 0), row_size=128, num_vals_limit=None):
    """In place on ``y``; reference src/common/row-op-util.hpp:101-119."""
    _rowop("oracle_assign_rows_from_double_index", y, x, index, offset, row_size, num_vals_limit)


def vs_add(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """y = a + b (mkl_alternate.hpp:59-74)."""
    y = np.empty_like(a)
    if lib().oracle_vs_add(a.size, _f(a), _f(b), _f(y)) != 0:
        raise ValueError("vsAdd precondition (n > 0) violated")
    return y


def apply_updates(master: np.ndarray, updates, threads: int = 1) -> None:
    """In place: for u in updates (arrival order): master = master + u
    (tablet-server.cpp:119-134 once per client message)."""
    arr = (_fp * max(1, len(updates)))(*[_f(u) for u in updates])
    for u in updates:
        assert u.size >= master.size
    if threads == 1:
        rc = lib().oracle_apply_updates(_f(master), arr, len(updates), master.size)
    else:
        rc = lib().oracle_apply_updates_mt(_f(master), arr, len(updates), master.size, threads)
    if rc != 0:
        raise ValueError(f"oracle_apply_updates failed ({rc})")


def server_partition(num_rows: int, num_servers: int):
    """(row_start[], num_rows[]) — clientlib-viter.cpp:674-682."""
    start = np.zeros(num_servers, dtype=np.uint64)
    count = np.zeros(num_servers, dtype=np.uint64)
    lib().oracle_server_partition(num_rows, num_servers, start.ctypes.data_as(_u64p),
                                  count.ctypes.data_as(_u64p))
    return start.astype(np.int64), count.astype(np.int64)


def synthetic_delta(client_id: int, num_vals: int) -> np.ndarray:
    """fp32 deltas uniform in [-0.5, 0.5), seed 1000 + client_id."""
    rng = np.random.default_rng(1000 + client_id)
    return (rng.random(num_vals, dtype=np.float32) - np.float32(0.5)).astype(np.float32)


def fill_uniform(out: np.ndarray, seed: int, threads: int = 1) -> np.ndarray:
    """Fill a float32 array with uniform [-0.5, 0.5) values, multi-threaded
    (synthetic deltas for the full-size CPU baseline; bench.py)."""
    assert out.dtype == np.float32 and out.flags.c_contiguous
    if lib().oracle_fill_uniform(_f(out), out.size, seed, threads) != 0:
        raise RuntimeError("oracle_fill_uniform failed")
    return out
