"""``shift_cuda``-compatible native-op module over the C ABI.

Same function names, argument meaning, return types and error behaviour as the
reference's pybind extension (``model/Temporal_shift/cuda/shift_cuda.cpp:19-47``):

* ``forward(input, xpos, ypos, stride) -> Tensor`` — ``input`` must be a contiguous device
  tensor (``CHECK_INPUT``, RuntimeError otherwise); ``ypos`` is the value the reference
  glue passes, i.e. ALREADY +0.5-shifted for stride != 1 (``shift.py:17-18``);
* ``backward(grad_output, input, output, xpos, ypos, stride) -> [gin, gx, gy]`` —
  ``grad_output`` and ``output`` checked like the reference (``shift_cuda.cpp:33-34``).

With ``sys.modules["shift_cuda"] = shiftgcn.shift_cuda`` the reference's unchanged
``cuda/shift.py`` runs its ``ShiftFunction`` on the gfx950 kernels.
"""
import torch

from . import ops
from . import torch_ops  # noqa: F401  (registers torch.ops.shiftgcn.*)


def forward(input, xpos, ypos, stride):  # noqa: A002 (reference names)
    ops.check_input(input, "input", input.dtype)
    return torch.ops.shiftgcn.tshift_fwd(input, xpos, ypos, stride, False)


def backward(grad_output, input, output, xpos, ypos, stride):  # noqa: A002
    ops.check_input(grad_output, "grad_output", grad_output.dtype)
    ops.check_input(output, "output", output.dtype)
    gin, gx, gy = torch.ops.shiftgcn.tshift_bwd(grad_output, input, xpos, ypos, stride, False)
    return [gin, gx, gy]
