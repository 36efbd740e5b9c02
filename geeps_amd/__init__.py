"""geeps_amd — MI355X-native GeePS gradient-update reduction path.

Product code:
  * geeps_amd/csrc/gp_kernels.hpp  HIP kernels (gfx950); gp_reduce.hip, gp_unplanned.hip,
                                   gp_runtime.hip, gp_host.cpp: the C-ABI (include/gp_reduce.h)
  * geeps_amd/csrc/geeps/          C++ drop-in libgeeps (include/geeps.hpp)
  * geeps_amd/native.py            ctypes binding of the C-ABI
  * geeps_amd/rowops.py            reference-named row ops / N-way sum on tensors
  * geeps_amd/shard.py             row-range sharding over ranks (RCCL exchange)

Nothing here imports oracle/ — that is test infrastructure.
"""
from .native import GpError, DoubleIndex, lib  # noqa: F401

__all__ = ["GpError", "DoubleIndex", "lib"]
