"""Scalar-loop restatement of the reference temporal-shift kernels (TEST INFRASTRUCTURE ONLY).

A second, deliberately naive restatement used to pin :mod:`oracle.shift_oracle`:
one Python loop iteration per CUDA thread, following
``model/Temporal_shift/cuda/shift_cuda_kernel.cu`` line by line with ``numpy.float32``
scalars (one rounding per operation). Small inputs only (pure-Python speed).
"""
from __future__ import annotations

import math

import numpy as np

F = np.float32


def _floorf_int(v) -> int:
    return int(math.floor(float(F(v))))


def _c_mod(a: int, b: int) -> int:
    """C++ ``%``: remainder truncated toward zero."""
    return int(math.fmod(a, b))


def _c_div(a: int, b: int) -> int:
    """C++ integer ``/``: quotient truncated toward zero."""
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b > 0) else -q


def forward(inp, xpos, ypos, stride):
    """``shift_cuda_forward_kernel`` (.cu:11-76), one iteration per thread ``index``."""
    B, C, Hb, Wb = inp.shape
    Ht, Wt = Hb // stride, Wb
    out = np.zeros((B, C, Ht, Wt), F)
    flat_in = inp.reshape(-1)
    for index in range(B * C * Ht * Wt):
        top_sp = Ht * Wt
        bot_sp = Hb * Wb
        n = index // (C * top_sp)
        idx = index % (C * top_sp)
        c = idx // top_sp
        sp = idx % top_sp
        h = sp // Wt
        w = sp % Wt
        base = n * C * bot_sp + c * bot_sp
        h_off = h * stride
        x = F(xpos[c])
        y = F(ypos[c])
        x1 = _floorf_int(x)
        x2 = x1 + 1
        y1 = _floorf_int(y)
        y2 = y1 + 1

        def tap(hi, wi):
            if hi >= 0 and wi >= 0 and hi < Hb and wi < Wb:
                return F(flat_in[base + hi * Wb + wi])
            return F(0)

        q11 = tap(h_off + y1, w + x1)
        q21 = tap(h_off + y1, w + x2)
        q12 = tap(h_off + y2, w + x1)
        q22 = tap(h_off + y2, w + x2)
        dx = F(x - F(x1))
        dy = F(y - F(y1))
        one = F(1)
        val = F(F(F(q11 * F(one - dx)) * F(one - dy)) + F(F(q21 * dx) * F(one - dy)))
        val = F(val + F(F(q12 * F(one - dx)) * dy))
        val = F(val + F(F(q22 * dx) * dy))
        out.reshape(-1)[index] = val
    return out


def bottom_backward(gout, xpos, ypos, Hb, stride):
    """``Shift_Bottom_Backward_Stride1`` (.cu:78-152) / ``Shift_Bottom_Backward`` (.cu:155-256)."""
    B, C, Ht, Wt = gout.shape
    Wb = Wt
    gin = np.zeros((B, C, Hb, Wb), F)
    flat_g = gout.reshape(-1)
    for index in range(B * C * Hb * Wb):
        bot_sp = Hb * Wb
        top_sp = Ht * Wt
        n = index // (C * bot_sp)
        idx = index % (C * bot_sp)
        c = idx // bot_sp
        sp = idx % bot_sp
        hc = sp // Wb
        wc = sp % Wb
        base = n * C * top_sp + c * top_sp
        x = F(-F(xpos[c]))
        y = F(-F(ypos[c]))
        x1 = _floorf_int(x)
        x2 = x1 + 1
        y1 = _floorf_int(y)
        y2 = y1 + 1

        def tap(hi, wi):
            if stride == 1:
                if hi >= 0 and wi >= 0 and hi < Hb and wi < Wb:
                    return F(flat_g[base + hi * Wb + wi])
                return F(0)
            if _c_mod(hi, 2) == 0:
                hq = _c_div(hi, 2)
                if hq >= 0 and wi >= 0 and hq < Ht and wi < Wt:
                    return F(flat_g[base + hq * Wt + wi])
            return F(0)

        q11 = tap(hc + y1, wc + x1)
        q21 = tap(hc + y1, wc + x2)
        q12 = tap(hc + y2, wc + x1)
        q22 = tap(hc + y2, wc + x2)
        dx = F(x - F(x1))
        dy = F(y - F(y1))
        one = F(1)
        val = F(F(F(q11 * F(one - dx)) * F(one - dy)) + F(F(q21 * dx) * F(one - dy)))
        val = F(val + F(F(q12 * F(one - dx)) * dy))
        val = F(val + F(F(q22 * dx) * dy))
        gin.reshape(-1)[index] = val
    return gin


def position_backward(inp, gout, xpos, ypos, stride):
    """``Shift_Position_Backward`` (.cu:277-363): the two (B,C,Ho,W) temporaries."""
    B, C, Hb, Wb = inp.shape
    Ht, Wt = Hb // stride, Wb
    gxb = np.zeros((B, C, Ht, Wt), F)
    gyb = np.zeros((B, C, Ht, Wt), F)
    flat_in = inp.reshape(-1)
    flat_g = gout.reshape(-1)
    for index in range(B * C * Ht * Wt):
        top_sp = Ht * Wt
        bot_sp = Hb * Wb
        n = index // (C * top_sp)
        idx = index % (C * top_sp)
        c = idx // top_sp
        sp = idx % top_sp
        h = sp // Wt
        w = sp % Wt
        base = n * C * bot_sp + c * bot_sp
        sx = F(xpos[c])
        sy = F(ypos[c])
        ix1 = _floorf_int(sx)
        iy1 = _floorf_int(sy)
        dx = F(sx - F(ix1))
        dy = F(sy - F(iy1))
        h1 = h * stride + iy1
        h2 = h1 + 1
        w1 = w + ix1
        w2 = w1 + 1

        def tap(hi, wi):
            if hi >= 0 and wi >= 0 and hi < Hb and wi < Wb:
                return F(flat_in[base + hi * Wb + wi])
            return F(0)

        q11, q21, q12, q22 = tap(h1, w1), tap(h1, w2), tap(h2, w1), tap(h2, w2)
        one = F(1)
        vx = F(F(F(one - dy) * F(q21 - q11)) + F(dy * F(q22 - q12)))
        vy = F(F(F(one - dx) * F(q12 - q11)) + F(dx * F(q22 - q21)))
        g = F(flat_g[index])
        gxb.reshape(-1)[index] = F(vx * g)
        gyb.reshape(-1)[index] = F(vy * g)
    return gxb, gyb
