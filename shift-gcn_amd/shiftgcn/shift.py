"""Drop-in for ``model/Temporal_shift/cuda/shift.py`` (``from cuda.shift import Shift``).

Same names, constructor signature, parameter names and autograd contract as the
reference (``shift.py:9-46``); the native calls go to the gfx950 HIP library instead of
``shift_cuda``. There is no CPU path: a CPU tensor raises like the reference's
``CHECK_INPUT`` (``shift_cuda.cpp:15-17``).
"""
from __future__ import annotations

import torch
from torch.autograd import Function
from torch.nn import Module, Parameter

from . import torch_ops  # noqa: F401  (registers torch.ops.shiftgcn.tshift_fwd / _bwd)


class ShiftFunction(Function):
    """``ShiftFunction`` (shift.py:9-30).

    The reference adds 0.5 to ``ypos`` for stride != 1 (a new fp32 tensor) before the
    native call and saves that shifted value; here the same fp32 add happens inside the
    kernel (forward and backward), so the saved tensor is the raw parameter and no extra
    elementwise launch is spent. Gradients w.r.t. ``ypos`` are identical because
    d(ypos+0.5)/d(ypos) = 1.
    """

    @staticmethod
    def forward(ctx, input, xpos, ypos, stride=1):  # noqa: A002 (reference name)
        input = input.contiguous()
        output = torch.ops.shiftgcn.tshift_fwd(input, xpos.detach(), ypos.detach(), stride,
                                               True)
        ctx.save_for_backward(input, xpos, ypos)
        ctx.stride = stride
        return output

    @staticmethod
    def backward(ctx, grad_output):
        grad_output = grad_output.contiguous()
        input, xpos, ypos = ctx.saved_tensors
        gin, gx, gy = torch.ops.shiftgcn.tshift_bwd(grad_output, input, xpos.detach(),
                                                    ypos.detach(), ctx.stride, True)
        return gin, gx, gy, None


class Shift(Module):
    """``Shift(channel, stride, init_scale=3)`` (shift.py:32-46)."""

    def __init__(self, channel, stride, init_scale=3, device=None):
        super().__init__()
        self.stride = stride
        if device is None:
            device = "cuda" if torch.cuda.is_available() else "cpu"
        self.xpos = Parameter(torch.zeros(channel, device=device))
        self.ypos = Parameter(torch.zeros(channel, device=device))
        self.xpos.data.uniform_(-1e-8, 1e-8)
        self.ypos.data.uniform_(-init_scale, init_scale)

    def forward(self, input):  # noqa: A002
        return ShiftFunction.apply(input, self.xpos, self.ypos, self.stride)
