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
from . import ops


def forward(input, xpos, ypos, stride):  # noqa: A002 (reference names)
    ops.check_input(input, "input")
    return ops.tshift_fwd(input, xpos.contiguous(), ypos.contiguous(), stride,
                          ypos_is_raw=False)


def backward(grad_output, input, output, xpos, ypos, stride):  # noqa: A002
    ops.check_input(grad_output, "grad_output")
    ops.check_input(output, "output")
    gin, gx, gy = ops.tshift_bwd(grad_output, input.contiguous(), xpos.contiguous(),
                                 ypos.contiguous(), stride, ypos_is_raw=False)
    return [gin, gx, gy]
