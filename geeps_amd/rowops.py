"""Row operations and the server's N-way sum on device tensors.

Host-side mirror of the reference's row-op interface, same names and argument
meaning, each call one C-ABI launch (include/gp_reduce.h) on the caller's
current HIP stream:

=================================  ===============================================
this module                        reference
=================================  ===============================================
add_rows_from_double_index_gpu     src/common/row-op-util.hpp:151-155 / .cu:109-142
assign_rows_to_double_index_gpu    src/common/row-op-util.hpp:141-145 / .cu:39-72
assign_rows_from_double_index_gpu  src/common/row-op-util.hpp:146-150 / .cu:74-107
add_row_batch_gpu                  src/common/row-op-util.hpp:72-79 (y += x)
gpu_add                            cpu_add, src/common/gpu-util/math_functions.hpp:60-61
zerofy_data_gpu                    DataStorage::zerofy_data_gpu, common-util.hpp:445-456
apply_updates                      TabletStorage::apply_updates x N in arrival order,
                                   src/server/tablet-server.cpp:119-134
gather_rows_segmented              assign_rows_to_double_index_gpu over a param cache
                                   split into row-range buffers (libgeeps in-place refreshes)
add_rows_segmented                 add_rows_from_double_index_gpu into such a cache
                                   (read-my-writes, clientlib-data.cpp:387-392)
RowPlan.add / RowPlan.init         add_rows_from_double_index_gpu (+ zerofy) over an
                                   index compiled once (vi_create_double_index,
                                   clientlib-viter.cpp:817-883), rows in cache order
=================================  ===============================================

Differences from the reference (deliberate, documented in DESIGN.md): launches
are asynchronous (the reference syncs after each, row-op-util.cu:141); sizes are
64-bit; errors raise ``GpError`` instead of aborting.

Tensors: values are float32 CUDA tensors addressed as flat arrays of
``row_size``-float rows; a DoubleIndex is an int64 CUDA tensor of shape (n, 2)
holding (id0, id1) per row.
"""
from __future__ import annotations

import ctypes
from typing import Sequence

import torch

from . import native
from .native import DoubleIndex, check

ROW_DATA_SIZE = 128  # include/geeps-user-defined-types.hpp


def _stream_ptr(stream) -> int:
    if stream is None:
        stream = torch.cuda.current_stream()
    return int(stream.cuda_stream) if hasattr(stream, "cuda_stream") else int(stream)


def _dev_f32(t: torch.Tensor, name: str) -> None:
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise ValueError(f"{name} must be a CUDA (HIP) tensor")
    if t.dtype != torch.float32:
        raise ValueError(f"{name} must be float32, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


def _as_offset(off) -> DoubleIndex:
    if off is None:
        return DoubleIndex(0, 0)
    if isinstance(off, DoubleIndex):
        return off
    a, b = off
    return DoubleIndex(int(a), int(b))


def _row_op(kind: str, rows_y, rows_x, index, num_rows, index_offset, row_size,
            num_vals_limit, stream, validate) -> None:
    _dev_f32(rows_y, "rows_y")
    _dev_f32(rows_x, "rows_x")
    if num_rows is None:
        num_rows = 0 if index is None else int(index.shape[0])
    if num_rows == 0:
        return
    if not (index.is_cuda and index.dtype == torch.int64 and index.dim() == 2
            and index.shape[1] == 2 and index.is_contiguous()):
        raise ValueError("index must be a contiguous int64 CUDA tensor of shape (n, 2)")
    if num_rows > index.shape[0]:
        raise ValueError("num_rows exceeds index length")
    if row_size <= 0:
        raise ValueError("row_size must be positive")
    off = _as_offset(index_offset)
    if num_vals_limit is None:
        num_vals_limit = (1 << 64) - 1
    if validate:
        _validate_bounds(kind, rows_y, rows_x, index[:num_rows], off, row_size, num_vals_limit)
    fn = {"add_from": native.lib().gp_scatter_add_rows,
          "init_from": native.lib().gp_scatter_init_rows,
          "assign_to": native.lib().gp_gather_rows,
          "assign_from": native.lib().gp_scatter_rows}[kind]
    check(fn(rows_y.data_ptr(), rows_x.data_ptr(), index.data_ptr(), num_rows, off,
             row_size, num_vals_limit, _stream_ptr(stream)), f"gp row op {kind}")


def _validate_bounds(kind, y, x, index, off, row_size, limit) -> None:
    """Host-side check that every access the kernel will make is in bounds.

    Mirrors the reference guard: rows whose guarded element index is past
    ``num_vals_limit`` are skipped element-wise, so only guarded-in elements
    are checked.  One device reduction + one sync.
    """
    if index.numel() == 0:
        return
    if int(index.min()) < 0:
        raise ValueError("negative row id in DoubleIndex")
    r0 = index[:, 0] + off.id0
    r1 = index[:, 1] + off.id1
    if kind == "assign_to":      # from = id1 (x), to = id0 (y), guard on y
        x_rows, y_rows, guarded = r1, r0, r0
    else:                        # from = id0 (x), to = id1 (y), guard on x
        x_rows, y_rows, guarded = r0, r1, r0
    if limit < (1 << 62):
        active = guarded * row_size < limit   # row touches >= 1 element
        if not bool(active.any()):
            return
        x_rows, y_rows = x_rows[active], y_rows[active]
    x_max, y_max = int(x_rows.max()), int(y_rows.max())
    x_need, y_need = (x_max + 1) * row_size, (y_max + 1) * row_size
    # The guarded side is touched only below the limit.
    if kind == "assign_to":
        y_need = min(y_need, limit)
    else:
        x_need = min(x_need, limit)
    if x_need > x.numel():
        raise ValueError(f"source row {x_max} out of range for rows_x")
    if y_need > y.numel():
        raise ValueError(f"destination row {y_max} out of range for rows_y")


def add_rows_from_double_index_gpu(rows_y, rows_x, index, num_rows=None, index_offset=None,
                                   row_size=ROW_DATA_SIZE, num_vals_limit=None,
                                   stream=None, validate=True) -> None:
    """``y[(id1+off1)*W + v] += x[(id0+off0)*W + v]`` where ``(id0+off0)*W+v < limit``.

    The client delta accumulate (reference row-op-util.cu:109-142).  Destination
    rows must be distinct within one call (as for the reference kernel).
    """
    _row_op("add_from", rows_y, rows_x, index, num_rows, index_offset, row_size,
            num_vals_limit, stream, validate)


def init_rows_from_double_index_gpu(rows_y, rows_x, index, num_rows=None, index_offset=None,
                                    row_size=ROW_DATA_SIZE, num_vals_limit=None,
                                    stream=None, validate=True) -> None:
    """Fused ``zerofy_data_gpu`` + ``add_rows_from_double_index_gpu`` for the
    listed destination rows: ``y[id1] = 0.0f + x[id0]`` (0.0f where guarded out)."""
    _row_op("init_from", rows_y, rows_x, index, num_rows, index_offset, row_size,
            num_vals_limit, stream, validate)


def assign_rows_to_double_index_gpu(rows_y, rows_x, index, num_rows=None, index_offset=None,
                                    row_size=ROW_DATA_SIZE, num_vals_limit=None,
                                    stream=None, validate=True) -> None:
    """``y[(id0+off0)*W + v] = x[(id1+off1)*W + v]`` where ``(id0+off0)*W+v < limit``."""
    _row_op("assign_to", rows_y, rows_x, index, num_rows, index_offset, row_size,
            num_vals_limit, stream, validate)


def assign_rows_from_double_index_gpu(rows_y, rows_x, index, num_rows=None, index_offset=None,
                                      row_size=ROW_DATA_SIZE, num_vals_limit=None,
                                      stream=None, validate=True) -> None:
    """``y[(id1+off1)*W + v] = x[(id0+off0)*W + v]`` where ``(id0+off0)*W+v < limit``."""
    _row_op("assign_from", rows_y, rows_x, index, num_rows, index_offset, row_size,
            num_vals_limit, stream, validate)


class RowPlan:
    """A DoubleIndex compiled once.  ``kind="scatter"`` (gp_row_plan_create):
    the rows in destination (id1) order; id0/id1-contiguous runs of >= 4 MiB
    moved by the phase-separated sum kernels, the rest by the wave-map row
    kernel over an id1-sorted device index.  ``kind="gather"``
    (gp_gather_plan_create): the same for assign_rows_to_double_index_gpu's
    index, in destination (id0) order, dense runs copied by the
    phase-separated kernels.

    ``index``: (n, 2) int64 array or tensor (copied to the host once);
    ``index_offset`` and ``num_vals_limit`` are baked in.  Scatter plans:
    ``add(y, x)`` / ``init(y, x)`` are bit-identical to
    add_rows_from_double_index_gpu / init_rows_from_double_index_gpu over the
    same index.  Gather plans: ``gather(y, x)`` / ``gather_segmented(y,
    segments)`` to assign_rows_to_double_index_gpu / gather_rows_segmented.
    A repeated destination is handled in op order through the plan's repeat
    layers (its adds in the order listed; for a gather the last one wins), as
    the reference's CPU twins loop (row-op-util.hpp:81-139)."""

    def __init__(self, index, num_rows=None, index_offset=None, row_size=ROW_DATA_SIZE,
                 num_vals_limit=None, kind="scatter"):
        if kind not in ("scatter", "gather"):
            raise ValueError("kind must be 'scatter' or 'gather'")
        self.kind = kind
        import numpy as np
        if isinstance(index, torch.Tensor):
            index = index.detach().cpu().numpy()
        idx = np.ascontiguousarray(index, dtype=np.int64)
        if idx.ndim != 2 or idx.shape[1] != 2:
            raise ValueError("index must have shape (n, 2)")
        n = idx.shape[0] if num_rows is None else int(num_rows)
        if n > idx.shape[0]:
            raise ValueError("num_rows exceeds index length")
        if n and int(idx[:n].min()) < 0:
            raise ValueError("negative row id in DoubleIndex")
        if row_size <= 0:
            raise ValueError("row_size must be positive")
        idx = np.ascontiguousarray(idx[:n])
        self.num_rows, self.row_size = n, int(row_size)
        self.offset = _as_offset(index_offset)
        self.limit = (1 << 64) - 1 if num_vals_limit is None else int(num_vals_limit)
        r0 = idx[:, 0] + self.offset.id0 if n else idx[:, 0]
        r1 = idx[:, 1] + self.offset.id1 if n else idx[:, 1]
        active = r0 * self.row_size < self.limit if self.limit < (1 << 62) else np.ones(n, bool)
        if kind == "scatter":
            # bounds the row kernels need: source rows below the limit, every destination
            self.x_need = min((int(r0[active].max()) + 1) * self.row_size, self.limit) if active.any() else 0
            self.y_need = (int(r1.max()) + 1) * self.row_size if n else 0
        else:
            # destinations (id0) below the limit, and whole source rows for them
            self.y_need = min((int(r0[active].max()) + 1) * self.row_size, self.limit) if active.any() else 0
            self.x_need = (int(r1[active].max()) + 1) * self.row_size if active.any() else 0
            self._src_rows = r1[active]
        self._h = ctypes.c_void_p()
        create = native.lib().gp_row_plan_create if kind == "scatter" else native.lib().gp_gather_plan_create
        check(create(ctypes.byref(self._h), idx.ctypes.data, n, self.offset, self.row_size, self.limit),
              "gp_row_plan_create" if kind == "scatter" else "gp_gather_plan_create")

    def info(self) -> dict:
        a, b, c = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
        check(native.lib().gp_row_plan_info(self._h, ctypes.byref(a), ctypes.byref(b),
                                            ctypes.byref(c)), "gp_row_plan_info")
        layers, rep = ctypes.c_size_t(), ctypes.c_size_t()
        check(native.lib().gp_row_plan_repeats(self._h, ctypes.byref(layers), ctypes.byref(rep)),
              "gp_row_plan_repeats")
        return {"rows": a.value, "dense_runs": b.value, "dense_rows": c.value,
                "residual_rows": a.value - c.value - rep.value, "repeat_layers": layers.value,
                "repeat_rows": rep.value}

    def launches(self, init: bool = False) -> dict:
        """Launch plan of one planned add (or fused init) over 16-B-aligned
        buffers: sweep / tile-major phased sum launches over the dense runs,
        and the rest (mixed / scalar sum forms, the residual's row kernel)."""
        a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(native.lib().gp_row_plan_launches(self._h, int(bool(init)), ctypes.byref(a),
                                                ctypes.byref(b), ctypes.byref(c)),
              "gp_row_plan_launches")
        return {"sweep": a.value, "phased": b.value, "other": c.value}

    def _run(self, fn, y, x, stream, what, kind="scatter"):
        if self.kind != kind:
            raise ValueError(f"a {self.kind} plan cannot run {what}")
        _dev_f32(y, "rows_y")
        _dev_f32(x, "rows_x")
        if self.x_need > x.numel():
            raise ValueError("source row out of range for rows_x")
        if self.y_need > y.numel():
            raise ValueError("destination row out of range for rows_y")
        check(fn(y.data_ptr(), x.data_ptr(), self._h, _stream_ptr(stream)), what)

    def add(self, rows_y, rows_x, stream=None) -> None:
        self._run(native.lib().gp_scatter_add_rows_planned, rows_y, rows_x, stream,
                  "gp_scatter_add_rows_planned")

    def init(self, rows_y, rows_x, stream=None) -> None:
        self._run(native.lib().gp_scatter_init_rows_planned, rows_y, rows_x, stream,
                  "gp_scatter_init_rows_planned")

    def gather(self, rows_y, rows_x, stream=None) -> None:
        self._run(native.lib().gp_gather_rows_planned, rows_y, rows_x, stream,
                  "gp_gather_rows_planned", kind="gather")

    def gather_segmented(self, rows_y, segments, stream=None) -> None:
        """``segments`` = [(first_row, tensor), ...] as for gather_rows_segmented."""
        if self.kind != "gather":
            raise ValueError("a scatter plan cannot run gp_gather_rows_segmented_planned")
        _dev_f32(rows_y, "rows_y")
        t, ranges = _segments(segments, self.row_size)
        if self.y_need > rows_y.numel():
            raise ValueError("destination row out of range for rows_y")
        if self.num_rows:
            src = getattr(self, "_src_rows_dev", None)
            if src is None or src.device != rows_y.device:  # copied to the device once
                src = self._src_rows_dev = torch.as_tensor(self._src_rows, device=rows_y.device)
            _validate_segment_rows(src, ranges)
        check(native.lib().gp_gather_rows_segmented_planned(rows_y.data_ptr(), ctypes.byref(t), self._h,
                                                            _stream_ptr(stream)),
              "gp_gather_rows_segmented_planned")

    def close(self) -> None:
        if self._h:
            native.lib().gp_row_plan_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _segments(segments, row_size):
    """[(first_row, tensor), ...] -> (RowSegments, row ranges) with checks."""
    if not 1 <= len(segments) <= native.GP_MAX_SEGMENTS:
        raise ValueError(f"1..{native.GP_MAX_SEGMENTS} segments required")
    t = native.RowSegments()
    t.count = len(segments)
    ranges = []
    for i, (first, buf) in enumerate(segments):
        _dev_f32(buf, f"segments[{i}]")
        first = int(first)
        if i == 0 and first != 0:
            raise ValueError("segments[0] must start at row 0")
        if i and first <= ranges[-1][0]:
            raise ValueError("segment first rows must ascend")
        t.first_row[i] = first
        t.base[i] = buf.data_ptr()
        ranges.append((first, buf.numel() // row_size))
    return t, ranges


def _validate_segment_rows(rows: torch.Tensor, ranges) -> None:
    """Every cache row maps into its segment's buffer."""
    if rows.numel() == 0:
        return
    firsts = torch.tensor([f for f, _ in ranges], device=rows.device, dtype=torch.int64)
    sizes = torch.tensor([n for _, n in ranges], device=rows.device, dtype=torch.int64)
    seg = torch.searchsorted(firsts, rows, right=True) - 1
    if bool(((rows - firsts[seg]) >= sizes[seg]).any()):
        raise ValueError("cache row past the end of its segment buffer")


def gather_rows_segmented(rows_y, segments, index, num_rows=None, index_offset=None,
                          row_size=ROW_DATA_SIZE, num_vals_limit=None, stream=None,
                          validate=True) -> None:
    """``assign_rows_to_double_index_gpu`` reading a segmented cache:
    ``segments`` = [(first_row, tensor), ...]; cache row c of the segment
    starting at f is row c - f of its tensor."""
    _dev_f32(rows_y, "rows_y")
    t, ranges = _segments(segments, row_size)
    n = int(index.shape[0]) if num_rows is None else int(num_rows)
    if n == 0:
        return
    off = _as_offset(index_offset)
    limit = (1 << 64) - 1 if num_vals_limit is None else int(num_vals_limit)
    if validate:
        idx = index[:n]
        to = idx[:, 0] + off.id0
        active = to * row_size < limit
        _validate_segment_rows((idx[:, 1] + off.id1)[active], ranges)
        if bool(active.any()) and min((int(to[active].max()) + 1) * row_size, limit) > rows_y.numel():
            raise ValueError("destination row out of range for rows_y")
    check(native.lib().gp_gather_rows_segmented(rows_y.data_ptr(), ctypes.byref(t), index.data_ptr(),
                                                n, off, row_size, limit, _stream_ptr(stream)),
          "gp_gather_rows_segmented")


def add_rows_segmented(segments, rows_x, index, num_rows=None, index_offset=None,
                       row_size=ROW_DATA_SIZE, num_vals_limit=None, stream=None,
                       validate=True) -> None:
    """``add_rows_from_double_index_gpu`` into a segmented cache."""
    _dev_f32(rows_x, "rows_x")
    t, ranges = _segments(segments, row_size)
    n = int(index.shape[0]) if num_rows is None else int(num_rows)
    if n == 0:
        return
    off = _as_offset(index_offset)
    limit = (1 << 64) - 1 if num_vals_limit is None else int(num_vals_limit)
    if validate:
        idx = index[:n]
        frm = idx[:, 0] + off.id0
        active = frm * row_size < limit
        _validate_segment_rows((idx[:, 1] + off.id1)[active], ranges)
        if bool(active.any()) and min((int(frm[active].max()) + 1) * row_size, limit) > rows_x.numel():
            raise ValueError("source row out of range for rows_x")
    check(native.lib().gp_scatter_add_rows_segmented(ctypes.byref(t), rows_x.data_ptr(),
                                                     index.data_ptr(), n, off, row_size, limit,
                                                     _stream_ptr(stream)),
          "gp_scatter_add_rows_segmented")


def bucket_sum_apply(master: torch.Tensor, buckets: Sequence[torch.Tensor],
                     num_vals: int | None = None, stream=None) -> None:
    """``master += b[0]; master += b[1]; ...`` in one pass, bit-identical to the
    sequential form (tablet-server.cpp:119-134 once per client, in order)."""
    _dev_f32(master, "master")
    n = master.numel() if num_vals is None else int(num_vals)
    if n > master.numel():
        raise ValueError("num_vals exceeds master size")
    ptrs = (ctypes.c_void_p * max(1, len(buckets)))()
    for k, b in enumerate(buckets):
        _dev_f32(b, f"buckets[{k}]")
        if b.numel() < n:
            raise ValueError(f"buckets[{k}] smaller than num_vals")
        if b.device != master.device:
            raise ValueError("bucket on a different device than master")
        ptrs[k] = b.data_ptr()
    check(native.lib().gp_bucket_sum_apply(master.data_ptr(), ptrs, len(buckets), n,
                                           _stream_ptr(stream)), "gp_bucket_sum_apply")


def bucket_sum_into(out: torch.Tensor, master: torch.Tensor, buckets: Sequence[torch.Tensor],
                    num_vals: int | None = None, stream=None) -> None:
    """``out = ((master + b[0]) + b[1]) + ...`` with ``master`` left unchanged:
    the next version of a shard built beside the published one (gp_bucket_sum_into)."""
    _dev_f32(master, "master")
    _dev_f32(out, "out")
    n = master.numel() if num_vals is None else int(num_vals)
    if n > master.numel() or n > out.numel():
        raise ValueError("num_vals exceeds master / out size")
    ptrs = (ctypes.c_void_p * max(1, len(buckets)))()
    for k, b in enumerate(buckets):
        _dev_f32(b, f"buckets[{k}]")
        if b.numel() < n:
            raise ValueError(f"buckets[{k}] smaller than num_vals")
        if b.device != master.device or out.device != master.device:
            raise ValueError("buffers on different devices")
        ptrs[k] = b.data_ptr()
    check(native.lib().gp_bucket_sum_into(out.data_ptr(), master.data_ptr(), ptrs, len(buckets), n,
                                          _stream_ptr(stream)), "gp_bucket_sum_into")


def apply_updates(master: torch.Tensor, updates: Sequence[torch.Tensor], stream=None) -> None:
    """The server's N-way sum: the reference's per-message ``apply_updates`` for
    each update in arrival order, as one device pass."""
    bucket_sum_apply(master, updates, stream=stream)


def gpu_add(n: int, a: torch.Tensor, b: torch.Tensor, y: torch.Tensor, stream=None) -> None:
    """``y[i] = a[i] + b[i]`` for i < n (cpu_add / vsAdd on the device)."""
    for t, nm in ((a, "a"), (b, "b"), (y, "y")):
        _dev_f32(t, nm)
        if t.numel() < n:
            raise ValueError(f"{nm} smaller than n")
    check(native.lib().gp_add(int(n), a.data_ptr(), b.data_ptr(), y.data_ptr(),
                              _stream_ptr(stream)), "gp_add")


def add_row_batch_gpu(rows_y: torch.Tensor, rows_x: torch.Tensor, batch_size: int,
                      row_size: int = ROW_DATA_SIZE, stream=None) -> None:
    """``y += x`` over ``batch_size`` rows (reference row-op-util.hpp:72-79)."""
    gpu_add(batch_size * row_size, rows_y, rows_x, rows_y, stream)


def zerofy_data_gpu(t: torch.Tensor, stream=None) -> None:
    _dev_f32(t, "t")
    check(native.lib().gp_zero(t.data_ptr(), t.numel(), _stream_ptr(stream)), "gp_zero")


# -- host-memory rows (the reference's CPU twins; libgeeps' host tier) ------
def _host_f32(a, name):
    import numpy as np
    if not (isinstance(a, np.ndarray) and a.dtype == np.float32 and a.flags.c_contiguous):
        raise ValueError(f"{name} must be a C-contiguous float32 numpy array")


def _host_index(index):
    import numpy as np
    if not (isinstance(index, np.ndarray) and index.dtype in (np.int64, np.uint64) and index.ndim == 2
            and index.shape[1] == 2 and index.flags.c_contiguous):
        raise ValueError("index must be a contiguous (n, 2) int64 numpy array")


def _host_bounds(kind, y, x, index, off, row_size, limit) -> None:
    """The host twins' bounds check, as _validate_bounds for the device ops:
    every element the C-ABI call will touch must lie inside the numpy arrays
    (the C code trusts its pointers: an id past the end would write the
    Python process's heap).  Negative ids and offsets are refused, as are ids
    whose element index could not be formed in 63 bits; the guarded side
    (the source of add / init, the destination of the gather) is touched only
    below ``limit``, rows wholly past it not at all."""
    import numpy as np
    if row_size <= 0:
        raise ValueError("row_size must be positive")
    if limit < 0:
        raise ValueError("num_vals_limit must not be negative")
    if off.id0 < 0 or off.id1 < 0:  # (a ctypes c_uint64 wraps a negative int: caught by the size test below)
        raise ValueError("negative index offset")
    if index.shape[0] == 0:
        return
    if index.dtype == np.int64 and int(index.min()) < 0:
        raise ValueError("negative row id in DoubleIndex")
    ids = index.view(np.uint64)
    top = int(ids.max()) + max(int(off.id0), int(off.id1))
    if (top + 1) * row_size >= 1 << 63:
        raise ValueError(f"row id {top} out of range for any array of {row_size}-float rows")
    r0 = ids[:, 0] + np.uint64(off.id0)
    r1 = ids[:, 1] + np.uint64(off.id1)
    if kind == "gather":   # y[id0] = x[id1], guard on y
        x_rows, y_rows, guarded = r1, r0, r0
    else:                  # y[id1] (+)= x[id0], guard on x
        x_rows, y_rows, guarded = r0, r1, r0
    if limit < (1 << 63):
        active = guarded * np.uint64(row_size) < np.uint64(limit)  # the row touches >= 1 element
        if not bool(active.any()):
            return
        x_rows, y_rows = x_rows[active], y_rows[active]
    x_max, y_max = int(x_rows.max()), int(y_rows.max())
    x_need, y_need = (x_max + 1) * row_size, (y_max + 1) * row_size
    if kind == "gather":
        y_need = min(y_need, limit)
    else:
        x_need = min(x_need, limit)
    if x_need > x.size:
        raise ValueError(f"source row {x_max} out of range for rows_x")
    if y_need > y.size:
        raise ValueError(f"destination row {y_max} out of range for rows_y")


def add_rows_from_double_index_cpu(rows_y, rows_x, index, index_offset=None, row_size=ROW_DATA_SIZE,
                                   num_vals_limit=None) -> None:
    """``y[(id1+off1)*W + v] += x[(id0+off0)*W + v]`` in host memory, entries in
    order (reference row-op-util.hpp:121-139) -- gp_host_scatter_add_rows."""
    _host_f32(rows_y, "rows_y")
    _host_f32(rows_x, "rows_x")
    _host_index(index)
    limit = (1 << 64) - 1 if num_vals_limit is None else num_vals_limit
    _host_bounds("add", rows_y, rows_x, index, _as_offset(index_offset), row_size, limit)
    check(native.lib().gp_host_scatter_add_rows(rows_y.ctypes.data, rows_x.ctypes.data, index.ctypes.data,
                                                index.shape[0], _as_offset(index_offset), row_size, limit),
          "gp_host_scatter_add_rows")


def init_rows_from_double_index_cpu(rows_y, rows_x, index, index_offset=None, row_size=ROW_DATA_SIZE,
                                    num_vals_limit=None) -> None:
    """``y[(id1+off1)*W + v] = 0.0f + x[(id0+off0)*W + v]`` (0.0f past the limit)
    in host memory: zerofy_data_cpu of the destination rows + the reference's
    add (row-op-util.hpp:121-139), fused -- gp_host_scatter_init_rows."""
    _host_f32(rows_y, "rows_y")
    _host_f32(rows_x, "rows_x")
    _host_index(index)
    limit = (1 << 64) - 1 if num_vals_limit is None else num_vals_limit
    _host_bounds("init", rows_y, rows_x, index, _as_offset(index_offset), row_size, limit)
    check(native.lib().gp_host_scatter_init_rows(rows_y.ctypes.data, rows_x.ctypes.data, index.ctypes.data,
                                                 index.shape[0], _as_offset(index_offset), row_size, limit),
          "gp_host_scatter_init_rows")


def assign_rows_to_double_index_cpu(rows_y, rows_x, index, index_offset=None, row_size=ROW_DATA_SIZE,
                                    num_vals_limit=None) -> None:
    """``y[(id0+off0)*W + v] = x[(id1+off1)*W + v]`` in host memory (reference
    row-op-util.hpp:81-99) -- gp_host_gather_rows."""
    _host_f32(rows_y, "rows_y")
    _host_f32(rows_x, "rows_x")
    _host_index(index)
    limit = (1 << 64) - 1 if num_vals_limit is None else num_vals_limit
    _host_bounds("gather", rows_y, rows_x, index, _as_offset(index_offset), row_size, limit)
    check(native.lib().gp_host_gather_rows(rows_y.ctypes.data, rows_x.ctypes.data, index.ctypes.data,
                                           index.shape[0], _as_offset(index_offset), row_size, limit),
          "gp_host_gather_rows")


def add_row_batch_cpu(rows_y, rows_x) -> None:
    """``y += x`` in host memory (reference add_row_batch, row-op-util.hpp:64-70) -- gp_host_add."""
    _host_f32(rows_y, "rows_y")
    _host_f32(rows_x, "rows_x")
    if rows_x.size < rows_y.size:
        raise ValueError("rows_x shorter than rows_y")
    check(native.lib().gp_host_add(rows_y.size, rows_y.ctypes.data, rows_x.ctypes.data), "gp_host_add")
