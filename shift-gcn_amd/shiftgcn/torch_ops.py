"""Dispatcher registration of the temporal shift (SURVEY §8b "a thin TORCH_LIBRARY layer").

The reference exposes its native op as the pybind module ``shift_cuda``
(``shift_cuda.cpp:44-47``), invisible to the dispatcher. Here the same two entry points are
registered as PyTorch operators over the C ABI, with fake (meta) kernels for shape
inference and the autograd formula attached, so ``torch.compile`` / ``torch.export`` /
FakeTensor tracing see them as single ops:

* ``shiftgcn::tshift_fwd(Tensor input, Tensor xpos, Tensor ypos, int stride,
  bool ypos_is_raw=False) -> Tensor`` — ``shift_cuda.forward`` (``shift_cuda.cpp:19-23``);
* ``shiftgcn::tshift_bwd(Tensor grad_output, Tensor input, Tensor xpos, Tensor ypos,
  int stride, bool ypos_is_raw=False) -> (Tensor, Tensor, Tensor)`` —
  ``shift_cuda.backward`` (``shift_cuda.cpp:25-42``; the unused ``output`` argument of the
  reference is dropped).

``ypos_is_raw=False`` is the reference glue's convention (``ypos`` already +0.5 for
stride != 1, ``shift.py:17-18``); ``True`` applies that fp32 add inside the kernel (what
``Shift`` uses). float32 and float64 (the reference's AT_DISPATCH_FLOATING_TYPES). There is
no CPU kernel: CPU tensors raise ``must be a CUDA tensor`` like ``CHECK_INPUT``.
"""
from __future__ import annotations

from typing import Tuple

import torch
from torch import Tensor

from . import ops


@torch.library.custom_op("shiftgcn::tshift_fwd", mutates_args=())
def tshift_fwd(input: Tensor, xpos: Tensor, ypos: Tensor, stride: int,  # noqa: A002
               ypos_is_raw: bool = False) -> Tensor:
    ops.check_input(input, "input", input.dtype)
    return ops.tshift_fwd(input, xpos.contiguous(), ypos.contiguous(), stride,
                          ypos_is_raw=ypos_is_raw)


@tshift_fwd.register_fake
def _tshift_fwd_fake(input, xpos, ypos, stride, ypos_is_raw=False):  # noqa: A002
    B, C, H, W = input.shape
    return input.new_empty((B, C, H // stride, W))


@torch.library.custom_op("shiftgcn::tshift_bwd", mutates_args=())
def tshift_bwd(grad_output: Tensor, input: Tensor, xpos: Tensor, ypos: Tensor,  # noqa: A002
               stride: int, ypos_is_raw: bool = False) -> Tuple[Tensor, Tensor, Tensor]:
    ops.check_input(grad_output, "grad_output", grad_output.dtype)
    return ops.tshift_bwd(grad_output, input.contiguous(), xpos.contiguous(),
                          ypos.contiguous(), stride, ypos_is_raw=ypos_is_raw)


@tshift_bwd.register_fake
def _tshift_bwd_fake(grad_output, input, xpos, ypos, stride, ypos_is_raw=False):  # noqa: A002
    C = input.shape[1]
    return input.new_empty(input.shape), input.new_empty((C,)), input.new_empty((C,))


def _setup_context(ctx, inputs, output):
    input, xpos, ypos, stride, ypos_is_raw = inputs  # noqa: A001
    ctx.save_for_backward(input, xpos, ypos)
    ctx.stride, ctx.ypos_is_raw = stride, ypos_is_raw


def _backward(ctx, grad_output):
    input, xpos, ypos = ctx.saved_tensors  # noqa: A001
    gin, gx, gy = torch.ops.shiftgcn.tshift_bwd(grad_output.contiguous(), input, xpos.detach(),
                                                ypos.detach(), ctx.stride, ctx.ypos_is_raw)
    return gin, gx, gy, None, None


tshift_fwd.register_autograd(_backward, setup_context=_setup_context)
