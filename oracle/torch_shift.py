"""Torch-eager, device-agnostic restatement of the reference temporal shift (TEST
INFRASTRUCTURE ONLY: the full-size parity tests run it on the GPU beside the HIP path, and
bench.py's cpu_baseline runs the oracle model with it on the host cores — BASELINE
config 1's "naive torch.gather temporal-shift fallback").

It is ``shift_cuda_kernel.cu`` written with whole-tensor gathers (the "naive torch.gather
temporal-shift fallback" of BASELINE config 1), on whatever device/dtype its inputs have:

* forward  (.cu:11-76): four taps at (h*stride + floor(y) + {0,1}, w + floor(x) + {0,1}),
  zero outside, blended ``q11(1-dx)(1-dy) + q21 dx(1-dy) + q12(1-dx)dy + q22 dx dy``;
* input gradient (.cu:78-256): the same blend of grad_output at the reversed position
  (stride 2: a tap lands only for an even row index, C++ remainder/quotient);
* position gradient (.cu:277-363, 501-509): val_x*g and val_y*g, mean over the batch,
  sum over W then H; ``applyShiftConstraint`` (.cu:370-395): +-0.01 / 0 (1e-4 if zero).

Same arithmetic as ``oracle/shift_oracle.py`` but in torch (no bit-exactness claimed: torch
may contract or reorder); used as the full-size eager reference of the model.
"""
from __future__ import annotations

import torch


def _frac(pos):
    i1 = torch.floor(pos.float()).long()
    return i1, pos - i1.to(pos.dtype)


def _taps(plane, hh, ww):
    """plane (B,C,H,W); hh (C,Ho,1), ww (C,1,W) long -> (B,C,Ho,W), zero outside."""
    B, C, H, W = plane.shape
    hh, ww = torch.broadcast_tensors(hh, ww)
    valid = (hh >= 0) & (ww >= 0) & (hh < H) & (ww < W)
    if H == 0:
        return plane.new_zeros((B, C) + tuple(hh.shape[1:]))
    hc, wc = hh.clamp(0, H - 1), ww.clamp(0, W - 1)
    cidx = torch.arange(C, device=plane.device)[:, None, None]
    out = plane[:, cidx, hc, wc]
    return torch.where(valid[None], out, torch.zeros((), dtype=plane.dtype, device=plane.device))


def _taps_s2(gout, hh, ww):
    B, C, Ht, W = gout.shape
    hh, ww = torch.broadcast_tensors(hh, ww)
    even = torch.fmod(hh, 2) == 0
    hq = torch.div(hh, 2, rounding_mode="trunc")
    valid = even & (hq >= 0) & (ww >= 0) & (hq < Ht) & (ww < W)
    if Ht == 0:
        return gout.new_zeros((B, C) + tuple(hh.shape[1:]))
    hc, wc = hq.clamp(0, Ht - 1), ww.clamp(0, W - 1)
    cidx = torch.arange(C, device=gout.device)[:, None, None]
    out = gout[:, cidx, hc, wc]
    return torch.where(valid[None], out, torch.zeros((), dtype=gout.dtype, device=gout.device))


def _blend(q11, q21, q12, q22, dx, dy):
    return q11 * (1 - dx) * (1 - dy) + q21 * dx * (1 - dy) + q12 * (1 - dx) * dy + q22 * dx * dy


def _grid(n, scale, off, dev):
    return torch.arange(n, device=dev)[None, :, None] * scale + off[:, None, None]


def shift_forward(inp, xpos, ypos, stride):
    B, C, H, W = inp.shape
    Ho = H // stride
    dev = inp.device
    x1, dx = _frac(xpos.to(inp.dtype))
    y1, dy = _frac(ypos.to(inp.dtype))
    h1 = _grid(Ho, stride, y1, dev)
    w1 = torch.arange(W, device=dev)[None, None, :] + x1[:, None, None]
    q = [_taps(inp, h1 + a, w1 + b) for a, b in ((0, 0), (0, 1), (1, 0), (1, 1))]
    return _blend(q[0], q[1], q[2], q[3], dx[None, :, None, None], dy[None, :, None, None])


def shift_backward(gout, inp, xpos, ypos, stride):
    B, C, H, W = inp.shape
    Ho = H // stride
    dev = inp.device
    dt = inp.dtype
    # input gradient: reversed shift of grad_output over the bottom grid
    rx1, rdx = _frac(-xpos.to(dt))
    ry1, rdy = _frac(-ypos.to(dt))
    h1 = _grid(H, 1, ry1, dev)
    w1 = torch.arange(W, device=dev)[None, None, :] + rx1[:, None, None]
    tap = _taps if stride == 1 else _taps_s2
    q = [tap(gout, h1 + a, w1 + b) for a, b in ((0, 0), (0, 1), (1, 0), (1, 1))]
    gin = _blend(q[0], q[1], q[2], q[3], rdx[None, :, None, None], rdy[None, :, None, None])
    # position gradients over the top grid
    x1, dx = _frac(xpos.to(dt))
    y1, dy = _frac(ypos.to(dt))
    h1 = _grid(Ho, stride, y1, dev)
    w1 = torch.arange(W, device=dev)[None, None, :] + x1[:, None, None]
    q11, q21, q12, q22 = [_taps(inp, h1 + a, w1 + b) for a, b in ((0, 0), (0, 1), (1, 0), (1, 1))]
    dxb, dyb = dx[None, :, None, None], dy[None, :, None, None]
    vx = ((1 - dyb) * (q21 - q11) + dyb * (q22 - q12)) * gout
    vy = ((1 - dxb) * (q12 - q11) + dxb * (q22 - q21)) * gout
    Gx = vx.double().mean(0).sum(2).sum(1)
    Gy = vy.double().mean(0).sum(2).sum(1)
    dr = Gy.abs()
    nz = dr != 0
    safe = torch.where(nz, dr, torch.ones_like(dr))
    gx = torch.where(nz, Gx / safe * 0.0, torch.zeros_like(Gx)).to(dt)
    gy = torch.where(nz, Gy / safe * 0.01, torch.full_like(Gy, 1e-4)).to(dt)
    return gin, gx, gy


class TorchShiftFunction(torch.autograd.Function):
    """``shift.py:9-30`` with ``shift_cuda`` replaced by the torch restatement above."""

    @staticmethod
    def forward(ctx, inp, xpos, ypos, stride=1):
        inp = inp.contiguous()
        ypos_eff = ypos if stride == 1 else ypos + 0.5
        ctx.save_for_backward(inp, xpos, ypos_eff)
        ctx.stride = stride
        return shift_forward(inp, xpos.detach(), ypos_eff.detach(), stride)

    @staticmethod
    def backward(ctx, grad_out):
        inp, xpos, ypos_eff = ctx.saved_tensors
        gin, gx, gy = shift_backward(grad_out.contiguous(), inp, xpos.detach(),
                                     ypos_eff.detach(), ctx.stride)
        return gin, gx, gy, None
