"""Tensor-level wrappers over the C ABI (``include/shiftgcn.h``).

Each wrapper validates like the reference binding (``shift_cuda.cpp:15-17``:
``<name> must be a CUDA tensor`` / ``must be contiguous``, raised as RuntimeError),
allocates outputs/workspace from torch's caching allocator on the tensor's device, and
enqueues on torch's CURRENT stream (so hipGraph capture and multi-stream use work).
"""
from __future__ import annotations

import torch

from . import _lib

_F32 = torch.float32


def _ptr(t):
    return None if t is None else t.data_ptr()


def _stream(t: torch.Tensor):
    return torch.cuda.current_stream(t.device).cuda_stream


def check_input(t: torch.Tensor, name: str) -> None:
    """``CHECK_INPUT`` of shift_cuda.cpp:15-17 (+ dtype: the HIP path is fp32)."""
    if not t.is_cuda:
        raise RuntimeError(f"{name} must be a CUDA tensor")
    if not t.is_contiguous():
        raise RuntimeError(f"{name} must be contiguous")
    if t.dtype != _F32:
        raise RuntimeError(f"{name} must be float32 (got {t.dtype})")


def _opt(t, name):
    if t is not None:
        check_input(t, name)
    return t


# --------------------------------------------------------------------------------------
# temporal shift
# --------------------------------------------------------------------------------------
def tshift_fwd(inp, xpos, ypos, stride, scale=None, shift=None, stats=None, out=None):
    """Forward shift of ``inp`` (B,C,H,W) -> (B,C,H//stride,W). ``ypos`` is the RAW
    parameter (the +0.5 for stride != 1 is applied in-kernel). Optional fused
    per-channel input affine (scale, shift) and per-plane output moments ``stats``
    (B*C*2 floats)."""
    check_input(inp, "input")
    check_input(xpos, "xpos")
    check_input(ypos, "ypos")
    _opt(scale, "scale"), _opt(shift, "shift"), _opt(stats, "stats")
    B, C, H, W = inp.shape
    if out is None:
        out = torch.empty((B, C, H // stride, W), device=inp.device, dtype=_F32)
    lib = _lib.load()
    rc = lib.sgcn_tshift_fwd(_ptr(inp), _ptr(out), _ptr(xpos), _ptr(ypos), _ptr(scale),
                             _ptr(shift), _ptr(stats), B, C, H, W, stride, _stream(inp))
    _lib.check(rc, "sgcn_tshift_fwd")
    return out


def tshift_bwd(gout, inp, xpos, ypos, stride, scale=None, shift=None, relu_mask=False):
    """Backward shift: returns (grad_input, grad_xpos, grad_ypos)."""
    check_input(gout, "grad_output")
    check_input(inp, "input")
    check_input(xpos, "xpos")
    check_input(ypos, "ypos")
    _opt(scale, "scale"), _opt(shift, "shift")
    B, C, H, W = inp.shape
    lib = _lib.load()
    dev = inp.device
    gin = torch.empty_like(inp)
    gx = torch.empty((C,), device=dev, dtype=_F32)
    gy = torch.empty((C,), device=dev, dtype=_F32)
    nbytes = lib.sgcn_tshift_bwd_ws_bytes(B, C)
    ws = torch.empty((max(nbytes, 4) + 3) // 4, device=dev, dtype=_F32)
    rc = lib.sgcn_tshift_bwd(_ptr(gout), _ptr(inp), _ptr(xpos), _ptr(ypos), _ptr(scale),
                             _ptr(shift), int(bool(relu_mask)), _ptr(gin), _ptr(gx), _ptr(gy),
                             _ptr(ws), nbytes, B, C, H, W, stride, _stream(inp))
    _lib.check(rc, "sgcn_tshift_bwd")
    return gin, gx, gy
