"""ctypes binding of the C-ABI in include/gp_reduce.h.

The HIP path is the only path: if ``geeps_amd/lib/libgp_reduce.so`` is missing
or does not export every declared symbol, loading raises immediately — there is
no CPU fallback anywhere in the package.
"""
from __future__ import annotations

import ctypes
import os
import re
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libgp_reduce.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "gp_reduce.h")

GP_OK = 0
GP_ERR_INVALID = 1
GP_ERR_HIP = 2


ABI_VERSION = 16  # GP_ABI_VERSION in include/gp_reduce.h


class GpError(RuntimeError):
    """A C-ABI call returned a non-zero status."""


class DoubleIndex(ctypes.Structure):
    """``gp_double_index`` == reference ``DoubleIndex`` (src/common/row-op-util.hpp:40-44)."""

    _fields_ = [("id0", ctypes.c_uint64), ("id1", ctypes.c_uint64)]


GP_MAX_SEGMENTS = 64  # include/gp_reduce.h


class RowSegments(ctypes.Structure):
    """``gp_row_segments``: a param cache split over up to 64 row-range buffers."""

    _fields_ = [("count", ctypes.c_uint32), ("reserved", ctypes.c_uint32),
                ("first_row", ctypes.c_uint64 * GP_MAX_SEGMENTS),
                ("base", ctypes.c_void_p * GP_MAX_SEGMENTS)]


class SumPlan(ctypes.Structure):
    """``gp_sum_plan``: every launch of one bucket-sum pass, by kernel form."""

    _fields_ = [("sweep_launches", ctypes.c_int), ("sweep_reg_tiles", ctypes.c_int),
                ("small_sweep_launches", ctypes.c_int),
                ("phased_launches", ctypes.c_int), ("phased_reg_tiles", ctypes.c_int),
                ("other_launches", ctypes.c_int),
                ("sweep_burst_tiles", ctypes.c_int), ("small_sweep_burst_tiles", ctypes.c_int),
                ("sweep_tile_kib", ctypes.c_int)]


class UnplannedStats(ctypes.Structure):
    """``gp_unplanned_stats``: what the unplanned calls' planning did (ABI 12)."""

    _fields_ = [(n, ctypes.c_uint64) for n in ("scans", "steady_calls", "stale_drops", "inverse_plans",
                                                "sorted_plans", "ranges_plans")]


_c = ctypes
_vp = _c.c_void_p
_sz = _c.c_size_t
_i = _c.c_int
# name -> (restype, argtypes)
_SIGNATURES = {
    "gp_abi_version": (_i, []),
    "gp_last_error": (_c.c_char_p, []),
    "gp_set_unplanned_min_bytes": (_i, [_sz]),
    "gp_unplanned_cache_clear": (_i, []),
    "gp_unplanned_cache_entries": (_i, [_c.POINTER(_sz), _c.POINTER(_sz)]),
    "gp_set_unplanned_cache_bytes": (_i, [_sz]),
    "gp_unplanned_stats_get": (_i, [_c.POINTER(UnplannedStats)]),
    "gp_scatter_add_rows": (_i, [_vp, _vp, _vp, _sz, DoubleIndex, _sz, _sz, _vp]),
    "gp_gather_rows": (_i, [_vp, _vp, _vp, _sz, DoubleIndex, _sz, _sz, _vp]),
    "gp_scatter_rows": (_i, [_vp, _vp, _vp, _sz, DoubleIndex, _sz, _sz, _vp]),
    "gp_scatter_init_rows": (_i, [_vp, _vp, _vp, _sz, DoubleIndex, _sz, _sz, _vp]),
    "gp_row_plan_create": (_i, [_c.POINTER(_vp), _vp, _sz, DoubleIndex, _sz, _sz]),
    "gp_row_plan_destroy": (_i, [_vp]),
    "gp_row_plan_info": (_i, [_vp, _c.POINTER(_sz), _c.POINTER(_sz), _c.POINTER(_sz)]),
    "gp_row_plan_repeats": (_i, [_vp, _c.POINTER(_sz), _c.POINTER(_sz)]),
    "gp_row_plan_launches": (_i, [_vp, _i, _c.POINTER(_i), _c.POINTER(_i), _c.POINTER(_i)]),
    "gp_gather_plan_create": (_i, [_c.POINTER(_vp), _vp, _sz, DoubleIndex, _sz, _sz]),
    "gp_gather_rows_planned": (_i, [_vp, _vp, _vp, _vp]),
    "gp_gather_rows_segmented_planned": (_i, [_vp, _c.POINTER(RowSegments), _vp, _vp]),
    "gp_scatter_add_rows_planned": (_i, [_vp, _vp, _vp, _vp]),
    "gp_scatter_init_rows_planned": (_i, [_vp, _vp, _vp, _vp]),
    "gp_gather_rows_segmented": (_i, [_vp, _c.POINTER(RowSegments), _vp, _sz, DoubleIndex, _sz,
                                      _sz, _vp]),
    "gp_scatter_add_rows_segmented": (_i, [_c.POINTER(RowSegments), _vp, _vp, _sz, DoubleIndex,
                                           _sz, _sz, _vp]),
    "gp_bucket_sum_apply": (_i, [_vp, _c.POINTER(_vp), _i, _sz, _vp]),
    "gp_bucket_sum_into": (_i, [_vp, _vp, _c.POINTER(_vp), _i, _sz, _vp]),
    "gp_bucket_sum_plan": (_i, [_sz, _i, _c.POINTER(_i), _c.POINTER(_i)]),
    "gp_bucket_sum_sweep_plan": (_i, [_sz, _i, _c.POINTER(_i), _c.POINTER(_i), _c.POINTER(_i)]),
    "gp_bucket_sum_launch_plan": (_i, [_sz, _i, _c.POINTER(SumPlan)]),
    "gp_add": (_i, [_sz, _vp, _vp, _vp, _vp]),
    "gp_host_scatter_add_rows": (_i, [_vp, _vp, _vp, _sz, DoubleIndex, _sz, _sz]),
    "gp_host_scatter_init_rows": (_i, [_vp, _vp, _vp, _sz, DoubleIndex, _sz, _sz]),
    "gp_host_gather_rows": (_i, [_vp, _vp, _vp, _sz, DoubleIndex, _sz, _sz]),
    "gp_host_add": (_i, [_sz, _vp, _vp]),
    "gp_host_zero": (_i, [_sz, _vp]),
    "gp_zero": (_i, [_vp, _sz, _vp]),
    "gp_hbm_probe": (_i, [_i, _vp, _sz, _vp]),
    "gp_device_count": (_i, [_c.POINTER(_i)]),
    "gp_set_device": (_i, [_i]),
    "gp_get_device": (_i, [_c.POINTER(_i)]),
    "gp_malloc_device": (_i, [_c.POINTER(_vp), _sz]),
    "gp_malloc_device_shared": (_i, [_c.POINTER(_vp), _sz]),
    "gp_free_device": (_i, [_vp]),
    "gp_malloc_host": (_i, [_c.POINTER(_vp), _sz]),
    "gp_free_host": (_i, [_vp]),
    "gp_host_register": (_i, [_vp, _sz]),
    "gp_host_unregister": (_i, [_vp]),
    "gp_memcpy_async": (_i, [_vp, _vp, _sz, _vp]),
    "gp_memset_async": (_i, [_vp, _i, _sz, _vp]),
    "gp_stream_create": (_i, [_c.POINTER(_vp)]),
    "gp_stream_destroy": (_i, [_vp]),
    "gp_stream_synchronize": (_i, [_vp]),
    "gp_device_synchronize": (_i, []),
    "gp_event_create": (_i, [_c.POINTER(_vp)]),
    "gp_event_destroy": (_i, [_vp]),
    "gp_event_record": (_i, [_vp, _vp]),
    "gp_event_synchronize": (_i, [_vp]),
    "gp_event_elapsed_ms": (_i, [_c.POINTER(_c.c_float), _vp, _vp]),
    "gp_stream_wait_event": (_i, [_vp, _vp]),
    "gp_device_pci_bus_id": (_i, [_i, _c.c_char_p, _i]),
    "gp_ipc_get_handle": (_i, [_vp, _vp]),
    "gp_ipc_open_handle": (_i, [_c.POINTER(_vp), _vp]),
    "gp_ipc_close_handle": (_i, [_vp]),
    "gp_ipc_describe_handle": (_i, [_vp, _c.c_char_p, _i]),
    "gp_ipc_mismaps": (_i, [_c.POINTER(_i)]),
}

_lock = threading.Lock()
_lib = None


def declared_symbols(header: str = HEADER_PATH) -> list[str]:
    """Every ``gp_*`` function declared in include/gp_reduce.h."""
    with open(header) as f:
        text = f.read()
    return sorted(set(re.findall(r"^\s*(?:int|const char \*)\s*(gp_\w+)\s*\(", text, re.M)))


def lib() -> ctypes.CDLL:
    """Load libgp_reduce.so once; raise loudly if it is missing or incomplete."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"geeps_amd: HIP library not built: {LIB_PATH} is missing "
                "(run `python -c 'import __graft_entry__ as g; g.build()'`)")
        handle = ctypes.CDLL(LIB_PATH)
        for name, (restype, argtypes) in _SIGNATURES.items():
            fn = getattr(handle, name)  # AttributeError = missing export: loud
            fn.restype = restype
            fn.argtypes = argtypes
        if handle.gp_abi_version() != ABI_VERSION:
            raise ImportError("geeps_amd: libgp_reduce.so ABI version mismatch")
        _lib = handle
        return _lib


def unplanned_stats() -> dict:
    """gp_unplanned_stats_get as a dict (process-wide counters since start)."""
    st = UnplannedStats()
    check(lib().gp_unplanned_stats_get(ctypes.byref(st)), "gp_unplanned_stats_get")
    return {name: getattr(st, name) for name, _ in UnplannedStats._fields_}


def check(rc: int, what: str = "") -> None:
    if rc != GP_OK:
        msg = lib().gp_last_error().decode(errors="replace")
        raise GpError(f"{what or 'gp call'} failed (status {rc}): {msg}")
