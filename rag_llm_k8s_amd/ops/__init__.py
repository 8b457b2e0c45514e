"""Operator layer: gfx950 HIP kernels for GPU tensors, torch reference on CPU.

``native``    -- shape-checked ctypes entry points (GPU only, raise if the library is missing)
``reference`` -- fp32 torch oracles / CPU execution path
"""
from . import reference  # noqa: F401
from ._lib import available as native_available  # noqa: F401
from .reference import pack_gate_up, rope_tables  # noqa: F401
