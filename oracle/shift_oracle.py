"""CPU oracle for the learnable fractional temporal shift (TEST INFRASTRUCTURE ONLY).

This module is the parity checker for the HIP temporal-shift kernels. Only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import it, and only as the checker: the product path never routes through it.

It restates, term by term and in float32 with one rounding per operation (no
fused multiply-add), the reference CUDA extension
``model/Temporal_shift/cuda/shift_cuda_kernel.cu``:

* :func:`shift_forward`          <- ``shift_cuda_forward_kernel``      (.cu:11-76) + launcher (.cu:405-431)
* :func:`shift_bottom_backward`  <- ``Shift_Bottom_Backward_Stride1`` (.cu:78-152) and
                                   ``Shift_Bottom_Backward`` (stride 2, .cu:155-256)
* :func:`shift_position_backward`<- ``Shift_Position_Backward``       (.cu:277-363)
* :func:`reduce_position_grad`   <- ATen ``mean(0)``/``sum(2)``/``sum(1)`` (.cu:501-509)
* :func:`apply_shift_constraint` <- ``applyShiftConstraint``          (.cu:370-395)
* :func:`shift_backward`         <- ``shift_cuda_backward``           (.cu:433-523)

and the Python glue ``model/Temporal_shift/cuda/shift.py:9-30`` (``ypos + 0.5`` for
stride != 1, computed in float32, is applied by the caller exactly as there).

Index arithmetic (``floorf`` → int, bounds tests, C++ remainder/quotient for the
stride-2 bottom backward) is reproduced bit-exactly.

Parity pinning: the reference's CUDA extension cannot be built or run in this image
(nvcc absent; its binding does not compile against torch 2.10; the prebuilt .so is
CUDA 9 / sm_30 and is never loaded). This restatement is pinned by (a) a second,
independent scalar-loop restatement in :mod:`oracle.shift_loops` checked element by
element, (b) hand-derived known-answer vectors (integer shifts are exact
translations; the reference ``demo.py`` case), and (c) the exact-adjoint property of
the bottom backward, all in ``tests/test_oracle_shift.py``.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32


def _floor_int(v: np.ndarray) -> np.ndarray:
    """``int x1 = floorf(x)`` (.cu:49) on a float vector. ``floorf`` is the float function:
    a double ``x`` (the reference's AT_DISPATCH double instantiation, .cu:413) is rounded
    to float first."""
    return np.floor(v.astype(np.float32)).astype(np.int64)


def _taps(plane: np.ndarray, hh: np.ndarray, ww: np.ndarray) -> np.ndarray:
    """Gather ``plane[..., hh, ww]`` with zero outside [0,H)x[0,W) (.cu:56-68).

    plane: (B, C, H, W); hh: (C, Ho, 1) int; ww: (C, 1, Wo) int -> (B, C, Ho, Wo).
    """
    B, C, H, W = plane.shape
    hh_b, ww_b = np.broadcast_arrays(hh, ww)
    valid = (hh_b >= 0) & (ww_b >= 0) & (hh_b < H) & (ww_b < W)
    if H == 0 or W == 0:
        return np.zeros((B, C) + hh_b.shape[1:], plane.dtype)
    hc = np.clip(hh_b, 0, H - 1)
    wc = np.clip(ww_b, 0, W - 1)
    cidx = np.arange(C)[:, None, None]
    out = plane[:, cidx, hc, wc]
    return np.where(valid[None], out, plane.dtype.type(0)).astype(plane.dtype)


def _fma(a, b, c):
    """fma(a, b, c) in the operands' precision: the float32 product is exact in float64,
    the sum is rounded in float64 and then to float32 (a double rounding that can differ
    from a true fused multiply-add in the last bit of rare ties; the contracted variant is
    only used as a bound, never for bit-exact checks)."""
    dt = np.result_type(a, b, c)
    if dt == np.float64:
        return a * b + c            # no wider type to emulate with; bound use only
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(dt)


def _bilinear(q11, q21, q12, q22, dx, dy, contract=False):
    """``q11*(1-dx)*(1-dy) + q21*dx*(1-dy) + q12*(1-dx)*dy + q22*dx*dy`` (.cu:73),
    evaluated left to right in float32 (each product/sum rounded once).

    ``contract=True``: the FMA-contracted evaluation nvcc emits by default
    (``--fmad=true``): each ``+ (u*v)*w`` becomes ``fma(u*v, w, acc)``."""
    one = q11.dtype.type(1)
    omdx = one - dx
    omdy = one - dy
    t1 = (q11 * omdx) * omdy
    if contract:
        acc = _fma(q21 * dx, omdy, t1)
        acc = _fma(q12 * omdx, dy, acc)
        return _fma(q22 * dx, dy, acc).astype(q11.dtype)
    t2 = (q21 * dx) * omdy
    t3 = (q12 * omdx) * dy
    t4 = (q22 * dx) * dy
    return (((t1 + t2) + t3) + t4).astype(q11.dtype)


def _frac(pos: np.ndarray):
    """Per-channel integer/fractional split: ``x1=floorf(x); dx=x-x1`` (.cu:49-71)."""
    i1 = _floor_int(pos)
    d = (pos - i1.astype(pos.dtype)).astype(pos.dtype)
    return i1, d


def shift_forward(inp: np.ndarray, xpos: np.ndarray, ypos: np.ndarray, stride: int,
                  contract: bool = False) -> np.ndarray:
    """Forward temporal shift. ``ypos`` must already carry the +0.5 for stride != 1
    (``shift.py:17-18``). Output shape (B, C, H // stride, W) (.cu:408).
    ``contract``: FMA-contracted blend (see :func:`_bilinear`)."""
    inp = np.ascontiguousarray(inp)
    dt = inp.dtype
    B, C, H, W = inp.shape
    Ho = H // stride
    x1, dx = _frac(xpos.astype(dt))
    y1, dy = _frac(ypos.astype(dt))
    h = np.arange(Ho)[None, :, None] * stride                # h_offset = h*stride
    w = np.arange(W)[None, None, :]                          # w_offset = w
    hy1 = h + y1[:, None, None]
    hy2 = hy1 + 1
    wx1 = w + x1[:, None, None]
    wx2 = wx1 + 1
    q11 = _taps(inp, hy1, wx1)
    q21 = _taps(inp, hy1, wx2)
    q12 = _taps(inp, hy2, wx1)
    q22 = _taps(inp, hy2, wx2)
    dxb = dx[None, :, None, None]
    dyb = dy[None, :, None, None]
    return _bilinear(q11, q21, q12, q22, dxb, dyb, contract)


def _taps_stride2_top(gout: np.ndarray, hh: np.ndarray, ww: np.ndarray) -> np.ndarray:
    """Stride-2 bottom-backward tap (.cu:203-248): a tap is taken only when
    ``h_im % 2 == 0`` (C++ remainder: truncated toward zero), then ``h_im/2``
    (C++ quotient, truncated) is bounds-checked against the top grid."""
    B, C, Ht, Wt = gout.shape
    hh_b, ww_b = np.broadcast_arrays(hh, ww)
    if Ht == 0 or Wt == 0:
        return np.zeros((B, C) + hh_b.shape[1:], gout.dtype)
    even = np.fmod(hh_b, 2) == 0
    hq = np.trunc(hh_b / 2).astype(np.int64)
    valid = even & (hq >= 0) & (ww_b >= 0) & (hq < Ht) & (ww_b < Wt)
    hc = np.clip(hq, 0, Ht - 1)
    wc = np.clip(ww_b, 0, Wt - 1)
    cidx = np.arange(C)[:, None, None]
    out = gout[:, cidx, hc, wc]
    return np.where(valid[None], out, gout.dtype.type(0)).astype(gout.dtype)


def shift_bottom_backward(gout: np.ndarray, xpos: np.ndarray, ypos: np.ndarray,
                          H: int, stride: int, contract: bool = False) -> np.ndarray:
    """Input gradient: bilinear sample of ``grad_output`` at the reversed position
    ``(-xpos, -ypos)`` over the bottom grid (.cu:78-152 stride 1, .cu:155-256 stride 2)."""
    gout = np.ascontiguousarray(gout)
    dt = gout.dtype
    B, C, Ht, W = gout.shape
    x1, dx = _frac(-xpos.astype(dt))
    y1, dy = _frac(-ypos.astype(dt))
    h = np.arange(H)[None, :, None]
    w = np.arange(W)[None, None, :]
    hy1 = h + y1[:, None, None]
    hy2 = hy1 + 1
    wx1 = w + x1[:, None, None]
    wx2 = wx1 + 1
    if stride == 1:
        tap = _taps
    elif stride == 2:
        tap = _taps_stride2_top
    else:  # the reference hard-codes stride 2 in its non-unit branch (.cu:172-174)
        raise ValueError("reference backward supports stride 1 and 2 only")
    q11 = tap(gout, hy1, wx1)
    q21 = tap(gout, hy1, wx2)
    q12 = tap(gout, hy2, wx1)
    q22 = tap(gout, hy2, wx2)
    return _bilinear(q11, q21, q12, q22, dx[None, :, None, None], dy[None, :, None, None],
                     contract)


def shift_position_backward(inp: np.ndarray, gout: np.ndarray, xpos: np.ndarray,
                            ypos: np.ndarray, stride: int, contract: bool = False):
    """Per-output-element position gradients ``val_x*g`` and ``val_y*g`` (.cu:277-363).

    Returns the two (B, C, Ho, W) temporaries the reference materialises (.cu:480-481)."""
    inp = np.ascontiguousarray(inp)
    gout = np.ascontiguousarray(gout, dtype=inp.dtype)
    dt = inp.dtype
    one = dt.type(1)
    B, C, H, W = inp.shape
    Ho = H // stride
    ix1, dx = _frac(xpos.astype(dt))
    iy1, dy = _frac(ypos.astype(dt))
    h = np.arange(Ho)[None, :, None] * stride
    w = np.arange(W)[None, None, :]
    h1 = h + iy1[:, None, None]
    h2 = h1 + 1
    w1 = w + ix1[:, None, None]
    w2 = w1 + 1
    q11 = _taps(inp, h1, w1)
    q21 = _taps(inp, h1, w2)
    q12 = _taps(inp, h2, w1)
    q22 = _taps(inp, h2, w2)
    dxb = dx[None, :, None, None]
    dyb = dy[None, :, None, None]
    # val_x = (1-dy)*(q21-q11)+dy*(q22-q12); val_y = (1-dx)*(q12-q11)+dx*(q22-q21)  (.cu:343-344)
    if contract:   # nvcc --fmad=true: a*b + c*d -> fma(c, d, a*b)
        val_x = _fma(np.broadcast_to(dyb, q22.shape), q22 - q12, (one - dyb) * (q21 - q11))
        val_y = _fma(np.broadcast_to(dxb, q22.shape), q22 - q21, (one - dxb) * (q12 - q11))
        val_x, val_y = val_x.astype(dt), val_y.astype(dt)
    else:
        val_x = ((one - dyb) * (q21 - q11) + dyb * (q22 - q12)).astype(dt)
        val_y = ((one - dxb) * (q12 - q11) + dxb * (q22 - q21)).astype(dt)
    return (val_x * gout).astype(dt), (val_y * gout).astype(dt)


def reduce_position_grad(g_bchw: np.ndarray) -> np.ndarray:
    """``mean`` over batch, then ``sum`` over W, then ``sum`` over H (.cu:501-509).

    The reference's reduction order inside each ATen op is an implementation detail of
    ATen/CUDA; only the sign (and zero-ness) of the result is observable after
    :func:`apply_shift_constraint`. float64 accumulation keeps the sign robust."""
    g = g_bchw.astype(np.float64)
    return g.mean(axis=0).sum(axis=2).sum(axis=1).astype(g_bchw.dtype)


def apply_shift_constraint(gx: np.ndarray, gy: np.ndarray):
    """``applyShiftConstraint`` (.cu:370-395), including its float/double promotions:
    ``dr = sqrt(dy*dy)`` in float; ``dx/dr*0.0`` and ``dy/dr*0.01`` are float
    quotients times *double* literals, rounded to float on store; the ``dr == 0``
    branch stores ``0.0`` and ``0.0001`` (as float). (float64 inputs stay float64.)"""
    dt = np.float64 if gy.dtype == np.float64 else F32
    gx = gx.astype(dt)
    gy = gy.astype(dt)
    dr = np.sqrt((gy * gy).astype(dt)).astype(dt)
    nz = dr != 0
    safe = np.where(nz, dr, dt(1))
    qx = (gx / safe).astype(dt)
    qy = (gy / safe).astype(dt)
    out_x = np.where(nz, (qx.astype(np.float64) * 0.0).astype(dt), dt(0.0))
    out_y = np.where(nz, (qy.astype(np.float64) * 0.01).astype(dt), dt(0.0001))
    return out_x.astype(dt), out_y.astype(dt)


def shift_backward(gout: np.ndarray, inp: np.ndarray, xpos: np.ndarray, ypos: np.ndarray,
                   stride: int, contract: bool = False):
    """``shift_cuda_backward`` (.cu:433-523): returns ``(grad_input, grad_xpos, grad_ypos)``.
    ``ypos`` is the (possibly +0.5-shifted) value saved by the forward (``shift.py:21``).
    ``contract``: the FMA-contracted variant of .cu:73 / .cu:343-344 (nvcc's default)."""
    H = inp.shape[2]
    gin = shift_bottom_backward(gout, xpos, ypos, H, stride, contract)
    gxb, gyb = shift_position_backward(inp, gout, xpos, ypos, stride, contract)
    gx, gy = apply_shift_constraint(reduce_position_grad(gxb), reduce_position_grad(gyb))
    return gin, gx, gy


def effective_ypos(ypos: np.ndarray, stride: int) -> np.ndarray:
    """``ShiftFunction.forward``'s ``ypos = ypos + 0.5`` for stride != 1 (``shift.py:14-18``),
    a float32 add."""
    return ypos if stride == 1 else (ypos + ypos.dtype.type(0.5)).astype(ypos.dtype)
