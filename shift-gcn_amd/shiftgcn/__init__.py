"""shiftgcn — MI355X (gfx950) Shift-GCN hot path.

Drop-in module surface of the reference (``model/shift_gcn.py``,
``model/Temporal_shift/cuda/shift.py``) on hand-written HIP kernels
(``shift-gcn_amd/csrc``) behind the C ABI ``include/shiftgcn.h``.
"""
from .shift import Shift, ShiftFunction  # noqa: F401

__all__ = ["Shift", "ShiftFunction"]
