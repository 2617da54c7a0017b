"""shiftgcn — MI355X (gfx950) Shift-GCN hot path.

Drop-in module surface of the reference (``model/shift_gcn.py``,
``model/Temporal_shift/cuda/shift.py``) on hand-written HIP kernels
(``shift-gcn_amd/csrc``) behind the C ABI ``include/shiftgcn.h``.
"""
from .shift import Shift, ShiftFunction  # noqa: F401
from .shift_gcn import (Model, Shift_gcn, Shift_tcn, TCN_GCN_unit, bn_init,  # noqa: F401
                        conv_init, import_class, tcn)

__all__ = ["Shift", "ShiftFunction", "Model", "Shift_gcn", "Shift_tcn", "TCN_GCN_unit", "tcn",
           "import_class", "conv_init", "bn_init"]
