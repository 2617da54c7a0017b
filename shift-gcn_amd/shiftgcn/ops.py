"""Tensor-level wrappers over the C ABI (``include/shiftgcn.h``).

Each wrapper validates like the reference binding (``shift_cuda.cpp:15-17``:
``<name> must be a CUDA tensor`` / ``must be contiguous``, raised as RuntimeError),
allocates outputs/workspace from torch's caching allocator on the tensor's device, and
enqueues on torch's CURRENT stream (so hipGraph capture and multi-stream use work).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib

_F32 = torch.float32


def _ptr(t):
    if t is None:
        return None
    return t.data_ptr()


# --------------------------------------------------------------------------------------
# optional launch timing (bench.py roofline): HIP events around each C-ABI call
# --------------------------------------------------------------------------------------
class LaunchTimer:
    """Records (op, algorithmic flops, algorithmic bytes, start, end) for every C-ABI call
    made while active, with events on the stream the kernels are launched on."""

    def __init__(self, ops_filter=None, detail=False):
        self.ops_filter = ops_filter
        self.detail = detail      # key records by op + launch shape (tools/shape_breakdown.py)
        self.records = []

    def begin(self, op, flops, nbytes, device):
        if self.ops_filter is not None and op not in self.ops_filter:
            return None
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(torch.cuda.current_stream(device))
        return (op, flops, nbytes, e0, e1, device)

    def end(self, rec):
        if rec is None:
            return
        rec[4].record(torch.cuda.current_stream(rec[5]))
        self.records.append(rec[:5])

    def summary(self, peak_flops=157.3e12, peak_bytes=8.0e12):
        """{op: {launches, ms_total, flops, bytes, roof_ms}} (call after a device sync);
        roof_ms = sum over launches of max(flops / peak_flops, bytes / peak_bytes), the
        time each launch would take at its own roofline bound."""
        out = {}
        for op, fl, nb, e0, e1 in self.records:
            d = out.setdefault(op, {"launches": 0, "ms_total": 0.0, "flops": 0.0, "bytes": 0.0,
                                    "roof_ms": 0.0})
            d["launches"] += 1
            d["ms_total"] += e0.elapsed_time(e1)
            d["flops"] += fl
            d["bytes"] += nb
            d["roof_ms"] += 1e3 * max(fl / peak_flops, nb / peak_bytes)
        return out


_TIMER = None


def set_launch_timer(timer):
    global _TIMER
    _TIMER = timer


class _timed:
    __slots__ = ("rec",)

    def __init__(self, op, flops, nbytes, t, detail=None):
        if _TIMER is None:
            self.rec = None
            return
        if _TIMER.detail and detail is not None:
            op = f"{op} {detail}"
        self.rec = _TIMER.begin(op, flops, nbytes, t.device)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        if self.rec is not None:
            _TIMER.end(self.rec)
        return False


def _shp(t):
    return "x".join(map(str, t.shape))


# --------------------------------------------------------------------------------------
# gradient slots: a parameter registered here (shiftgcn.dist.GradAllReduce's flat bucket)
# gets its gradient written straight into its slot of the bucket, as a fresh view that
# autograd's AccumulateGrad takes as the parameter's .grad (it steals a gradient nothing
# else references), so the data-parallel step needs no gather of the gradients into the
# bucket and no copy back. Only while .grad is None: with an existing .grad (accumulation)
# the new gradient goes to fresh memory and autograd adds it into .grad as usual.
# --------------------------------------------------------------------------------------
from torch.utils.weak import WeakIdKeyDictionary  # noqa: E402

_GRAD_SLOTS = WeakIdKeyDictionary()


def register_grad_slots(named, flat):
    """Map every parameter of ``named`` ([(name, p)], bucket order) to its slot of the
    1-D ``flat`` fp32 bucket; returns the offsets."""
    offs, off = [], 0
    for _, p in named:
        _GRAD_SLOTS[p] = (flat, off)
        offs.append(off)
        off += p.numel()
    if off != flat.numel():
        raise ValueError("gradient bucket size does not match the parameters")
    return offs


def unregister_grad_slots(params):
    for p in params:
        _GRAD_SLOTS.pop(p, None)


def grad_slot(p):
    """A fresh view of p's bucket slot (p's shape), or None if p has no slot."""
    s = _GRAD_SLOTS.get(p)
    if s is None:
        return None
    flat, off = s
    return flat[off:off + p.numel()].view(p.shape)


def is_grad_slot(p, t):
    """Whether ``t`` is p's bucket slot (the same memory)."""
    s = _GRAD_SLOTS.get(p)
    return (s is not None and t.data_ptr() == s[0].data_ptr() + 4 * s[1] and
            t.numel() == p.numel())


# slots handed out since the bucket's last release (GradAllReduce.__call__): a slot goes to
# at most ONE gradient tensor per backward. A parameter with two gradient contributions in
# one backward (the model called twice before one backward), or two torch.autograd.grad
# calls, would otherwise get the same memory twice: the second kernel would overwrite the
# first contribution before autograd sums them.
_SLOT_TAKEN = WeakIdKeyDictionary()


def release_grad_slots(params):
    """Make the slots of ``params`` available to the next backward."""
    for p in params:
        _SLOT_TAKEN.pop(p, None)


def grad_like(p):
    """Output tensor for p's gradient: its bucket slot while p.grad is None and the slot was
    not handed out yet since the last release, else a new tensor like p."""
    if p.grad is None and p not in _SLOT_TAKEN:
        v = grad_slot(p)
        if v is not None:
            _SLOT_TAKEN[p] = True
            return v
    return torch.empty_like(p)


def bump_versions(tensors):
    """Advance the autograd version counters of tensors a HIP kernel wrote in place through
    a raw pointer (torch cannot see those writes): anything keyed on ``_version`` — the
    eval-mode caches below, fused.folded_conv_bn, autograd's saved-tensor checks — then
    sees the change."""
    ts = [t for t in tensors if t is not None]
    if ts:
        torch.autograd.graph.increment_version(ts)


def _src_key(tensors):
    return tuple((t.data_ptr(), t._version) if t is not None else None for t in tensors)


def _cache_tensors(v):
    if isinstance(v, BnStats):
        return (v.buf,)
    if isinstance(v, torch.Tensor):
        return (v,)
    return tuple(t for x in v for t in _cache_tensors(x))


# Set once a native writer of parameters or running statistics (FusedSGD.step, a training
# BatchNorm finalize) has been captured in a hipGraph: a replay of that graph rewrites them
# without advancing any version counter, so from then on the version-keyed eval caches
# below are not trusted — every call recomputes its constants (inside a capture that puts
# them into the graph, so a replayed eval reads current weights too).
_CAPTURED_WRITES = False


def mark_captured_writes():
    global _CAPTURED_WRITES
    _CAPTURED_WRITES = True


def cached(owner, slot, key, make, device):
    """Value computed by ``make()`` once per ``key`` (storage + version of every tensor it
    reads), kept in ``owner.__dict__[slot]``: the eval-mode constants (BatchNorm apply
    coefficients, tanh(Feature_Mask) + 1) that change only when a weight or running
    statistic does. A stream that reads a cached tensor other than the one that made it is
    recorded on it (the caching allocator then keeps its memory until that stream is done
    when the entry is replaced). Nothing is stored during a hipGraph capture (the value
    would stay unwritten until the first replay), and nothing is cached at all once a
    training step's writers were captured (mark_captured_writes)."""
    if _CAPTURED_WRITES:
        owner.__dict__.pop(slot, None)
        return make()
    c = owner.__dict__.get(slot)
    cur = torch.cuda.current_stream(device)
    capturing = torch.cuda.is_current_stream_capturing()
    if c is not None and c[0] == key:
        if cur not in c[2] and not capturing:
            for t in _cache_tensors(c[1]):
                t.record_stream(cur)
            c[2].add(cur)
        return c[1]
    v = make()
    if not capturing:
        owner.__dict__[slot] = (key, v, {cur})
    return v


def _stream(t: torch.Tensor):
    return torch.cuda.current_stream(t.device).cuda_stream


def check_input(t: torch.Tensor, name: str, dtype=_F32) -> None:
    """``CHECK_INPUT`` of shift_cuda.cpp:15-17 (+ dtype: the fused path is fp32; the plain
    temporal shift also takes float64, like the reference's AT_DISPATCH_FLOATING_TYPES)."""
    if not t.is_cuda:
        raise RuntimeError(f"{name} must be a CUDA tensor")
    if not t.is_contiguous():
        raise RuntimeError(f"{name} must be contiguous")
    if t.dtype != dtype:
        raise RuntimeError(f"{name} must be {dtype} (got {t.dtype})")


def _opt(t, name):
    if t is not None:
        check_input(t, name)
    return t


# --------------------------------------------------------------------------------------
# temporal shift
# --------------------------------------------------------------------------------------
def tshift_fwd(inp, xpos, ypos, stride, scale=None, shift=None, stats=None, out=None,
               ypos_is_raw=True, affine=None):
    """Forward shift of ``inp`` (B,C,H,W) -> (B,C,H//stride,W). ``ypos`` is the RAW
    parameter (the +0.5 for stride != 1 is applied in-kernel). Optional fused
    per-channel input affine (scale, shift) — or ``affine``, a BnStats supplying them — and
    per-plane output moments
    ``stats`` (B*C*2 floats). float64 tensors run the double-precision kernel (no fused
    options)."""
    if affine is not None:
        scale, shift = affine.scale, affine.shift
    if inp.dtype == torch.float64:
        if scale is not None or shift is not None or stats is not None:
            raise RuntimeError("the fused shift options are float32-only")
        return _tshift_fwd_f64(inp, xpos, ypos, stride, ypos_is_raw, out)
    check_input(inp, "input")
    check_input(xpos, "xpos")
    check_input(ypos, "ypos")
    _opt(scale, "scale"), _opt(shift, "shift"), _opt(stats, "stats")
    B, C, H, W = inp.shape
    if out is None:
        out = torch.empty((B, C, H // stride, W), device=inp.device, dtype=_F32)
    lib = _lib.load()
    nb = 4 * (inp.numel() + out.numel())
    with _timed("tshift_fwd", 0, nb, inp, _shp(inp)):
        rc = lib.sgcn_tshift_fwd(_ptr(inp), _ptr(out), _ptr(xpos), _ptr(ypos), _ptr(scale),
                                 _ptr(shift), _ptr(stats), B, C, H, W, stride,
                                 int(ypos_is_raw), _stream(inp))
    _lib.check(rc, "sgcn_tshift_fwd")
    return out


def _tshift_fwd_f64(inp, xpos, ypos, stride, ypos_is_raw, out=None):
    _F64 = torch.float64
    check_input(inp, "input", _F64)
    check_input(xpos, "xpos", _F64)
    check_input(ypos, "ypos", _F64)
    B, C, H, W = inp.shape
    if out is None:
        out = torch.empty((B, C, H // stride, W), device=inp.device, dtype=_F64)
    with _timed("tshift_fwd", 0, 8 * (inp.numel() + out.numel()), inp, _shp(inp)):
        rc = _lib.load().sgcn_tshift_fwd_f64(_ptr(inp), _ptr(out), _ptr(xpos), _ptr(ypos), B,
                                             C, H, W, stride, int(ypos_is_raw), _stream(inp))
    _lib.check(rc, "sgcn_tshift_fwd_f64")
    return out


def _tshift_bwd_f64(gout, inp, xpos, ypos, stride, ypos_is_raw):
    _F64 = torch.float64
    check_input(gout, "grad_output", _F64)
    check_input(inp, "input", _F64)
    check_input(xpos, "xpos", _F64)
    check_input(ypos, "ypos", _F64)
    B, C, H, W = inp.shape
    lib = _lib.load()
    dev = inp.device
    gin = torch.empty_like(inp)
    gx = torch.empty((C,), device=dev, dtype=_F64)
    gy = torch.empty((C,), device=dev, dtype=_F64)
    nbytes = lib.sgcn_tshift_bwd_f64_ws_bytes(B, C)
    ws = torch.empty((max(nbytes, 8) + 7) // 8, device=dev, dtype=_F64)
    with _timed("tshift_bwd", 0, 8 * (gout.numel() + 2 * inp.numel()), inp, _shp(inp)):
        rc = lib.sgcn_tshift_bwd_f64(_ptr(gout), _ptr(inp), _ptr(xpos), _ptr(ypos), _ptr(gin),
                                     _ptr(gx), _ptr(gy), _ptr(ws), nbytes, B, C, H, W, stride,
                                     int(ypos_is_raw), _stream(inp))
    _lib.check(rc, "sgcn_tshift_bwd_f64")
    return gin, gx, gy


TAIL_MAX_PLANE = 16384   # sgcn_tshift_fwd_tail / _pre: LDS-staged planes only


def tshift_fwd_pre(z, xpos, ypos, stride, zst, r, rst, ast):
    """Inference: shift(ast-affine(relu(per-joint zst-affine(z) + res))) in one launch;
    res = r or rst-affine(r). The Shift_gcn output H is never materialised."""
    check_input(z, "z")
    check_input(r, "residual")
    B, C, H, W = z.shape
    out = torch.empty((B, C, H // stride, W), device=z.device, dtype=_F32)
    nb = 4 * (2 * z.numel() + out.numel())
    with _timed("tshift_fwd", 0, nb, z, _shp(z)):
        rc = _lib.load().sgcn_tshift_fwd_pre(
            _ptr(z), _ptr(out), _ptr(xpos), _ptr(ypos), _ptr(zst.scale), _ptr(zst.shift),
            _ptr(r), _ptr(rst.scale) if rst else None, _ptr(rst.shift) if rst else None,
            _ptr(ast.scale), _ptr(ast.shift), B, C, H, W, stride, 1, _stream(z))
    _lib.check(rc, "sgcn_tshift_fwd_pre")
    return out


def tshift_fwd_tail(inp, xpos, ypos, stride, st, r=None, rst=None, gather_m=None):
    """Inference unit tail: relu(BN(shift(inp)) + res) in one launch with the eval-mode
    coefficients ``st``, + the next unit's gathered gcn input when ``gather_m`` is given.
    Returns (out, gathered|None)."""
    check_input(inp, "input")
    if r is not None:
        check_input(r, "residual")
    B, C, H, W = inp.shape
    out = torch.empty((B, C, H // stride, W), device=inp.device, dtype=_F32)
    og = torch.empty_like(out) if gather_m is not None else None
    nb = 4 * (inp.numel() + out.numel() * (1 + (r is not None) + (og is not None)))
    with _timed("tshift_fwd", 0, nb, inp, _shp(inp)):
        rc = _lib.load().sgcn_tshift_fwd_tail(
            _ptr(inp), _ptr(out), _ptr(xpos), _ptr(ypos), _ptr(st.scale), _ptr(st.shift),
            _ptr(r), _ptr(rst.scale) if rst else None, _ptr(rst.shift) if rst else None,
            _ptr(gather_m), _ptr(og), B, C, H, W, stride, 1, _stream(inp))
    _lib.check(rc, "sgcn_tshift_fwd_tail")
    return out, og


class PosPartials:
    """Per-plane position-gradient partials left by a shift backward called with
    ``defer_pos=True``; ``finalize(gx, gy)`` runs sgcn_tshift_pos_finalize on the current
    stream (e.g. a side stream: the positions' gradients only feed the optimizer)."""

    __slots__ = ("ws", "B", "C")

    def __init__(self, ws, B, C):
        self.ws, self.B, self.C = ws, B, C

    def finalize(self, gx, gy):
        check_input(gx, "gx")
        check_input(gy, "gy")
        with _timed("finalize", 0, self.ws.numel() * 4, self.ws):
            rc = _lib.load().sgcn_tshift_pos_finalize(_ptr(self.ws), self.B, self.C, _ptr(gx),
                                                      _ptr(gy), _stream(self.ws))
        _lib.check(rc, "sgcn_tshift_pos_finalize")
        return gx, gy


def _pos_out(defer_pos, ws, B, C, dev, pos_out=None):
    """(gx, gy) tensors for the kernel (``pos_out`` if given, e.g. gradient slots), or
    (None, None) + PosPartials when deferred."""
    if defer_pos:
        return None, None, PosPartials(ws, B, C)
    if pos_out is not None:
        for t, n in zip(pos_out, ("grad_xpos", "grad_ypos")):
            check_input(t, n)
            if t.numel() != C:
                raise ValueError(f"{n} must hold {C} elements")
        return pos_out[0], pos_out[1], None
    return (torch.empty((C,), device=dev, dtype=_F32), torch.empty((C,), device=dev, dtype=_F32),
            None)


def tshift_bwd(gout, inp, xpos, ypos, stride, scale=None, shift=None, relu_mask=False,
               ypos_is_raw=True, bn_stats=None, defer_pos=False, pos_out=None):
    """Backward shift: returns (grad_input, grad_xpos, grad_ypos), plus the BatchNorm
    backward partials of ``bn_stats`` (the BN whose output feeds the shift) if given.
    ``defer_pos``: grad_xpos is a PosPartials and grad_ypos None (see PosPartials).
    float64 tensors run the double-precision kernel (no fused options)."""
    if inp.dtype == torch.float64:
        if (scale is not None or shift is not None or relu_mask or bn_stats is not None):
            raise RuntimeError("the fused shift options are float32-only")
        return _tshift_bwd_f64(gout, inp, xpos, ypos, stride, ypos_is_raw)
    check_input(gout, "grad_output")
    check_input(inp, "input")
    check_input(xpos, "xpos")
    check_input(ypos, "ypos")
    _opt(scale, "scale"), _opt(shift, "shift")
    B, C, H, W = inp.shape
    lib = _lib.load()
    dev = inp.device
    gin = torch.empty_like(inp)
    nbytes = lib.sgcn_tshift_bwd_ws_bytes(B, C)
    ws = torch.empty((max(nbytes, 4) + 3) // 4, device=dev, dtype=_F32)
    gx, gy, pp = _pos_out(defer_pos, ws, B, C, dev, pos_out)
    bpart = torch.empty((B * C * 2,), device=dev, dtype=_F32) if bn_stats is not None else None
    nb = 4 * (gout.numel() + 2 * inp.numel())
    with _timed("tshift_bwd", 0, nb, inp, _shp(inp)):
        rc = lib.sgcn_tshift_bwd(_ptr(gout), _ptr(inp), _ptr(xpos), _ptr(ypos), _ptr(scale),
                                 _ptr(shift), int(bool(relu_mask)),
                                 _ptr(bn_stats.mean) if bn_stats is not None else None,
                                 _ptr(bn_stats.invstd) if bn_stats is not None else None,
                                 _ptr(bpart), _ptr(gin), _ptr(gx), _ptr(gy), _ptr(ws), nbytes,
                                 B, C, H, W, stride, int(ypos_is_raw), _stream(inp))
    _lib.check(rc, "sgcn_tshift_bwd")
    if pp is not None:
        gx = pp
    if bn_stats is not None:
        return gin, gx, gy, bpart
    return gin, gx, gy


GBN_MAX_PLANE = 16384    # sgcn_tshift_bwd_gbn: LDS-staged stride-1 planes only


def ra_fits(n, V):
    """Whether a stride-1 plane of n = T*V elements fits the joint-aligned LDS backward
    kernels (sgcn_tshift_bwd_bnin / _gbn): V <= 64, <= 32 elements per thread. bnin runs
    256 threads up to 4,096 floats and 512 above; gbn runs 256 up to 8,192 floats but
    takes 512 whenever 256 would need more than 32 elements per thread, so both launch
    every plane this accepts."""
    if V > 64 or n > GBN_MAX_PLANE:
        return False
    # the padded LDS plane (tshift.hip kPadRows zero rows each side, a zero column each
    # side, one spare float) within 64 KiB
    if (n // V + 2 * 4) * (V + 2) + 1 > 16384:
        return False
    nt = 256 if n <= 4096 else 512
    return -(-n // ((nt // V) * V)) <= 32


def tshift_bwd_gbn(gout, inp, xpos, ypos, st: "BnStats", z, zst: "BnStats", defer_pos=False,
                   down=None, pos_out=None):
    """Shift_tcn.shift_in backward (stride 1, Shift_tcn.bn's affine on the taps and its
    backward partials) that also emits the k-free backward sums of Shift_gcn.bn, whose
    input is ``z`` and whose ReLU output is ``inp`` (sgcn_tshift_bwd_gbn). ``down`` =
    (d, d_stats): the Shift_gcn's down conv output and its BatchNorm's statistics — the
    six plane sums of that BatchNorm's backward come out of the same launch. Returns
    (grad_input, grad_xpos, grad_ypos, bn_part, z_part6[, d_part6])."""
    check_input(gout, "grad_output")
    check_input(inp, "input")
    check_input(z, "z")
    if down is not None:
        check_input(down[0], "d")
    B, C, H, W = inp.shape
    lib = _lib.load()
    dev = inp.device
    gin = torch.empty_like(inp)
    nbytes = lib.sgcn_tshift_bwd_ws_bytes(B, C)
    ws = torch.empty((max(nbytes, 4) + 3) // 4, device=dev, dtype=_F32)
    gx, gy, pp = _pos_out(defer_pos, ws, B, C, dev, pos_out)
    bpart = torch.empty((B * C * 2,), device=dev, dtype=_F32)
    zpart = torch.empty((6 * B * C * W,), device=dev, dtype=_F32)
    d, dst, dpart = None, None, None
    if down is not None:
        d, dst = down
        dpart = torch.empty((6 * B * C,), device=dev, dtype=_F32)
    nb = 4 * (gout.numel() + (3 if down is None else 4) * inp.numel())
    with _timed("tshift_bwd", 0, nb, inp, ("GBND " if down is not None else "GBN ") + _shp(inp)):
        rc = lib.sgcn_tshift_bwd_gbn(_ptr(gout), _ptr(inp), _ptr(xpos), _ptr(ypos),
                                     _ptr(st.scale), _ptr(st.shift), _ptr(st.mean),
                                     _ptr(st.invstd), _ptr(bpart), _ptr(z), _ptr(zst.mean),
                                     _ptr(zst.invstd), _ptr(zpart), _ptr(d),
                                     _ptr(dst.mean if dst is not None else None),
                                     _ptr(dst.invstd if dst is not None else None),
                                     _ptr(dpart), _ptr(gin), _ptr(gx), _ptr(gy), _ptr(ws),
                                     nbytes, B, C, H, W, _stream(inp))
    _lib.check(rc, "sgcn_tshift_bwd_gbn")
    if down is not None:
        return gin, (pp if pp is not None else gx), gy, bpart, zpart, dpart
    return gin, (pp if pp is not None else gx), gy, bpart, zpart


BNIN_MAX_PLANE = 16384   # sgcn_tshift_bwd_bnin: LDS-staged stride-1 planes only


def tshift_bwd_bnin(dy, y, s, coef, inp, xpos, ypos, defer_pos=False, pos_out=None):
    """Stride-1 shift backward (ReLU mask on ``inp``) whose output gradient is the input
    gradient of the following BatchNorm, k1*(y > 0 ? dy : 0) + k2*s + k3 (s = that
    BatchNorm's input), formed in the kernel. Returns (grad_input, grad_xpos, grad_ypos)."""
    for t, n in ((dy, "dy"), (y, "y"), (s, "s"), (inp, "input"), (coef, "coef")):
        check_input(t, n)
    B, C, H, W = inp.shape
    lib = _lib.load()
    dev = inp.device
    gin = torch.empty_like(inp)
    nbytes = lib.sgcn_tshift_bwd_ws_bytes(B, C)
    ws = torch.empty((max(nbytes, 4) + 3) // 4, device=dev, dtype=_F32)
    gx, gy, pp = _pos_out(defer_pos, ws, B, C, dev, pos_out)
    nb = 4 * (3 * dy.numel() + 2 * inp.numel())
    with _timed("tshift_bwd", 0, nb, inp, _shp(inp)):
        rc = lib.sgcn_tshift_bwd_bnin(
            _ptr(dy), _ptr(y), _ptr(s), _ptr(coef), _ptr(inp), _ptr(xpos), _ptr(ypos),
            _ptr(gin), _ptr(gx), _ptr(gy), _ptr(ws), nbytes, B, C, H, W, 1, _stream(inp))
    _lib.check(rc, "sgcn_tshift_bwd_bnin")
    return gin, (pp if pp is not None else gx), gy


# --------------------------------------------------------------------------------------
# pointwise (1x1) contraction with fused joint-shift gathers
# --------------------------------------------------------------------------------------
class PlaneView:
    """Plane-operand addressing of include/shiftgcn.h: element (b, ch, n = t*V + v) at
    ``t.data[b*bstride + ch*cstride + (t*tstride)*V + (v + rsign*ch) mod V]``."""

    __slots__ = ("t", "bstride", "cstride", "tstride", "rsign")

    def __init__(self, t, tstride=1, rsign=0):
        check_input(t, "plane operand")
        self.t = t
        self.bstride = t.stride(0)
        self.cstride = t.stride(1)
        self.tstride = tstride
        self.rsign = rsign


# The contraction kernels address each operand through a 32-bit buffer descriptor: every
# plane operand's extent must stay below 2^29 elements (sgcn_pw_fwd / sgcn_pw_dw return
# SGCN_EINVAL otherwise, pwconv.hip). Larger batches (NTU l5 at > ~279 clips per GPU) are
# split over B here into chunks that fit; the result is identical (forward/dX: every output
# element is the same fixed-order sum) or the same deterministic split-K reduction
# accumulated chunk by chunk (dW).
PW_MAX_ELEMS = 1 << 29


def _plane_extent(v: PlaneView, B, C, T, V):
    return (B - 1) * v.bstride + C * v.cstride + T * v.tstride * V


def _batch_chunk(views, B, T, V):
    """Largest batch chunk whose every (view, channels) extent is < PW_MAX_ELEMS."""
    bc = B
    for v, C in views:
        per = v.bstride
        fixed = C * v.cstride + T * v.tstride * V
        if fixed >= PW_MAX_ELEMS:
            raise ValueError("pointwise operand plane too large for one sample")
        if (B - 1) * per + fixed >= PW_MAX_ELEMS:
            bc = min(bc, max(1, (PW_MAX_ELEMS - 1 - fixed) // max(per, 1) + 1))
    return bc


def pw_fwd(w, w_mcontig, bias, x: PlaneView, out: PlaneView, M, K, T, V, mask=None,
           relu=False, accumulate=False):
    check_input(w, "weight")
    _opt(bias, "bias"), _opt(mask, "mask")
    B = x.t.shape[0]
    lib = _lib.load()
    P = B * T * V
    bc = _batch_chunk([(x, K), (out, M)], B, T, V)
    det = (f"M{M} K{K} T{T} V{V} xrot{x.rsign} yrot{out.rsign} mask{int(mask is not None)} "
           f"ts{x.tstride}{out.tstride} acc{int(accumulate)} mc{int(w_mcontig)}")
    with _timed("pw_fwd", 2.0 * P * M * K, 4.0 * P * (M * (2 if accumulate else 1) + K), x.t,
                det):
        for b0 in range(0, B, bc):
            nb = min(bc, B - b0)
            rc = lib.sgcn_pw_fwd(_ptr(w), int(w_mcontig), _ptr(bias),
                                 x.t.data_ptr() + 4 * b0 * x.bstride, x.bstride,
                                 x.cstride, x.tstride, x.rsign, _ptr(mask),
                                 out.t.data_ptr() + 4 * b0 * out.bstride,
                                 out.bstride, out.cstride, out.tstride, out.rsign, int(relu),
                                 int(accumulate), nb, M, K, T, V, _stream(x.t))
            _lib.check(rc, "sgcn_pw_fwd")
    return out.t


def pw_dw(g: PlaneView, x: PlaneView, dw, M, Nc, T, V, mask=None, transpose=False,
          accumulate=False, dbias=None, dbias_accumulate=False):
    check_input(dw, "dw")
    _opt(dbias, "dbias"), _opt(mask, "mask")
    B = g.t.shape[0]
    lib = _lib.load()
    bc = _batch_chunk([(g, M), (x, Nc)], B, T, V)
    nbytes = lib.sgcn_pw_dw_ws_bytes(bc, M, Nc, T, V)
    ws = torch.empty((nbytes + 3) // 4, device=g.t.device, dtype=_F32)
    P = B * T * V
    det = (f"M{M} N{Nc} T{T} V{V} grot{g.rsign} xrot{x.rsign} mask{int(mask is not None)} "
           f"ts{g.tstride}{x.tstride}")
    with _timed("pw_dw", 2.0 * P * M * Nc, 4.0 * P * (M + Nc), g.t, det):
        for b0 in range(0, B, bc):
            nb = min(bc, B - b0)
            first = b0 == 0
            rc = lib.sgcn_pw_dw(g.t.data_ptr() + 4 * b0 * g.bstride, g.bstride, g.cstride,
                                g.tstride, g.rsign, x.t.data_ptr() + 4 * b0 * x.bstride,
                                x.bstride, x.cstride, x.tstride, x.rsign, _ptr(mask),
                                _ptr(dw), int(transpose), int(accumulate or not first),
                                _ptr(dbias), int(dbias_accumulate or not first), _ptr(ws),
                                nbytes, nb, M, Nc, T, V, _stream(g.t))
            _lib.check(rc, "sgcn_pw_dw")
    return dw


def pw_fwd_tshift(w, bias, x: PlaneView, xpos, ypos, st, out: PlaneView, M, K, T, V,
                  relu=False, x_shifted=None, two_row=2):
    """Shift_tcn's shift_in fused into temporal_linear (sgcn_pw_fwd_tshift):
    out = act(w @ shift(st.scale*x + st.shift) + bias); the shifted operand is formed while
    staging and never read back (``x_shifted``: optionally stored, layout of x, for the
    weight gradient). ``st``: the BnStats of Shift_tcn.bn (None = identity); w is (M, K)
    k-contiguous. ``two_row``: 0 = every channel from four taps (bit-identical to
    tshift_fwd); 1 = channels with xpos in (-2^-25, 0] from two taps of their own column
    (still bit-identical); 2 = also 0 < xpos < 2^-25 (within 3e-8 * max|tap|)."""
    check_input(w, "weight")
    _opt(bias, "bias")
    if x.tstride != 1 or x.rsign != 0 or out.tstride != 1 or out.rsign != 0:
        raise ValueError("pw_fwd_tshift: plain planes only")
    B = x.t.shape[0]
    lib = _lib.load()
    P = B * T * V
    nbytes = lib.sgcn_pw_tshift_ws_bytes(K)
    ws = torch.empty((nbytes + 3) // 4, device=x.t.device, dtype=_F32)
    bc = _batch_chunk([(x, K), (out, M)], B, T, V)
    sc = st.scale if st is not None else None
    sh = st.shift if st is not None else None
    if x_shifted is not None:
        check_input(x_shifted, "x_shifted")
        if x_shifted.shape != x.t.shape or x_shifted.stride() != x.t.stride():
            raise ValueError("x_shifted must have the layout of x")
    nbx = 4.0 * P * (M + K * (2 if x_shifted is not None else 1))
    with _timed("pw_fwd", 2.0 * P * M * K, nbx, x.t,
                f"TSH M{M} K{K} T{T} V{V} side{int(x_shifted is not None)}"):
        for b0 in range(0, B, bc):
            nb = min(bc, B - b0)
            xs = None if x_shifted is None else x_shifted.data_ptr() + 4 * b0 * x.bstride
            rc = lib.sgcn_pw_fwd_tshift(_ptr(w), _ptr(bias), x.t.data_ptr() + 4 * b0 * x.bstride,
                                        x.bstride, x.cstride, _ptr(xpos), _ptr(ypos), _ptr(sc),
                                        _ptr(sh), xs, _ptr(ws), nbytes,
                                        out.t.data_ptr() + 4 * b0 * out.bstride, out.bstride,
                                        out.cstride, int(relu), int(two_row), nb, M, K, T, V,
                                        _stream(x.t))
            _lib.check(rc, "sgcn_pw_fwd_tshift")
    return out.t


# --------------------------------------------------------------------------------------
# BatchNorm / unit tails
# --------------------------------------------------------------------------------------
def moments(x, per_joint):
    check_input(x, "input")
    B, C, T, V = x.shape
    part = torch.empty((B * C * (V if per_joint else 1) * 2,), device=x.device, dtype=_F32)
    with _timed("bn_stats", 0, 4 * x.numel(), x, _shp(x)):
        rc = _lib.load().sgcn_moments(_ptr(x), _ptr(part), B, C, T, V, int(per_joint),
                                      _stream(x))
    _lib.check(rc, "sgcn_moments")
    return part


class BnStats:
    """Statistics and apply coefficients of one BatchNorm call (local feature order):
    batch statistics in training mode, running statistics in eval mode (``batch``)."""

    __slots__ = ("mean", "invstd", "scale", "shift", "buf", "batch")

    def __init__(self, F, device, batch=True):
        buf = torch.empty((4, F), device=device, dtype=_F32)
        self.buf = buf
        self.mean, self.invstd, self.scale, self.shift = buf[0], buf[1], buf[2], buf[3]
        self.batch = batch


def bn_finalize(part, B, F, n_part, bn, perm_V=0, training=True):
    """Training-mode statistics of ``bn`` (an nn.BatchNorm*d) from partials; updates its
    running stats / num_batches_tracked exactly once, like ``bn.forward`` in train()."""
    st = BnStats(F, part.device)
    lib = _lib.load()
    track = training and bn.track_running_stats and bn.running_mean is not None
    if track and bn.momentum is None:
        # the cumulative moving average (momentum=None) is never used by the reference
        raise NotImplementedError("BatchNorm momentum=None is not supported on the HIP path")
    momentum = bn.momentum if bn.momentum is not None else 0.0
    with _timed("finalize", 0, 4 * part.numel(), part):
        rc = lib.sgcn_bn_finalize(
            _ptr(part), B, F, n_part, perm_V, _ptr(bn.weight), _ptr(bn.bias), float(bn.eps),
            float(momentum), _ptr(bn.running_mean) if track else None,
            _ptr(bn.running_var) if track else None,
            _ptr(bn.num_batches_tracked) if track else None, _ptr(st.mean),
            _ptr(st.invstd), _ptr(st.scale), _ptr(st.shift), _stream(part))
    _lib.check(rc, "sgcn_bn_finalize")
    if track:   # the running statistics were written in place by the kernel
        bump_versions((bn.running_mean, bn.running_var, bn.num_batches_tracked))
        if torch.cuda.is_current_stream_capturing():
            mark_captured_writes()
    return st


def bn_eval_coef(bn, F, perm_V=0, device=None):
    """Eval-mode coefficients of ``bn`` (running statistics), computed once per version of
    its weight, bias and running statistics (:func:`cached`; the training step's writers
    bump those versions: FusedSGD, bn_finalize, broadcast_buffers)."""
    key = _src_key((bn.weight, bn.bias, bn.running_mean, bn.running_var)) + (
        float(bn.eps), F, perm_V)
    return cached(bn, "_sgcn_eval_coef", key, lambda: _bn_eval_coef(bn, F, perm_V),
                  bn.running_mean.device)


def _bn_eval_coef(bn, F, perm_V):
    st = BnStats(F, bn.running_mean.device, batch=False)
    with _timed("finalize", 0, 4 * 8 * F, bn.running_mean):
        rc = _lib.load().sgcn_bn_eval_coef(F, perm_V, _ptr(bn.weight), _ptr(bn.bias),
                                           _ptr(bn.running_mean), _ptr(bn.running_var),
                                           float(bn.eps), _ptr(st.mean), _ptr(st.invstd),
                                           _ptr(st.scale), _ptr(st.shift),
                                           _stream(bn.running_mean))
    _lib.check(rc, "sgcn_bn_eval_coef")
    return st


def bn_apply(x, st: BnStats, per_joint, r=None, rst: BnStats = None, relu=False, out=None,
             out_stats=None, gather_m=None):
    """Returns y; with ``out_stats`` given (True/False) returns (y, moments of y or None);
    with ``gather_m`` returns (y, gcn_gather(y, gather_m)) from one launch."""
    check_input(x, "input")
    if r is not None:
        check_input(r, "residual")
    B, C, T, V = x.shape
    y = torch.empty_like(x) if out is None else out
    ys = torch.empty((B * C * 2,), device=x.device, dtype=_F32) if out_stats else None
    yg = torch.empty_like(y) if gather_m is not None else None
    nb = 4 * x.numel() * (2 + (r is not None) + (yg is not None))
    with _timed("bn_apply", 0, nb, x, _shp(x)):
        rc = _lib.load().sgcn_bn_apply(
            _ptr(x), _ptr(st.scale), _ptr(st.shift), int(per_joint), _ptr(r),
            _ptr(rst.scale) if rst is not None else None,
            _ptr(rst.shift) if rst is not None else None, int(relu), _ptr(y), _ptr(ys),
            _ptr(gather_m), _ptr(yg), B, C, T, V, _stream(x))
    _lib.check(rc, "sgcn_bn_apply")
    if gather_m is not None:
        return y, yg
    return y if out_stats is None else (y, ys)


def bn_bwd_reduce(dy, y, relu, x, st: BnStats, per_joint, r=None, rst: BnStats = None,
                  dy_coef=None):
    check_input(dy, "grad_output")
    B, C, T, V = x.shape
    dev = x.device
    part = torch.empty((B * C * (V if per_joint else 1) * 2,), device=dev, dtype=_F32)
    rpart = torch.empty((B * C * 2,), device=dev, dtype=_F32) if r is not None else None
    nb = 4 * x.numel() * (2 + (y is not None) + (r is not None))
    with _timed("bn_bwd_reduce", 0, nb, x, _shp(x)):
        rc = _lib.load().sgcn_bn_bwd_reduce(_ptr(dy), _ptr(y), int(relu), _ptr(x),
                                            _ptr(st.mean), _ptr(st.invstd), int(per_joint),
                                            _ptr(r), _ptr(rst.mean) if rst else None,
                                            _ptr(rst.invstd) if rst else None, _ptr(dy_coef),
                                            _ptr(part), _ptr(rpart), B, C, T, V, _stream(x))
    _lib.check(rc, "sgcn_bn_bwd_reduce")
    return part, rpart


def bn_bwd_finalize(part, B, F, n_total, st: BnStats, bn, perm_V=0):
    """Returns (coef[3,F], dgamma, dbeta) with dgamma/dbeta in the module's layout."""
    dev = part.device
    coef = torch.empty((3, F), device=dev, dtype=_F32)
    dgamma = grad_like(bn.weight) if bn.weight is not None else None
    dbeta = grad_like(bn.bias) if bn.bias is not None else None
    with _timed("finalize", 0, 4 * part.numel(), part):
        rc = _lib.load().sgcn_bn_bwd_finalize(_ptr(part), B, F, int(n_total), perm_V,
                                              _ptr(st.mean), _ptr(st.invstd), _ptr(bn.weight),
                                              _ptr(dgamma), _ptr(dbeta), 0, int(st.batch),
                                              _ptr(coef), _stream(part))
    _lib.check(rc, "sgcn_bn_bwd_finalize")
    return coef, dgamma, dbeta


def bn_bwd_finalize_gbn(part6, B, C, V, n_total, dy_coef, dy_st: BnStats, st: BnStats, bn):
    """sgcn_bn_bwd_finalize_gbn: the per-joint BatchNorm1d's (coef[3, C*V], dgamma, dbeta)
    from sgcn_tshift_bwd_gbn's sums and the following BatchNorm's coefficients/mean."""
    dev = part6.device
    F = C * V
    coef = torch.empty((3, F), device=dev, dtype=_F32)
    dgamma = grad_like(bn.weight) if bn.weight is not None else None
    dbeta = grad_like(bn.bias) if bn.bias is not None else None
    with _timed("finalize", 0, 4 * part6.numel(), part6):
        rc = _lib.load().sgcn_bn_bwd_finalize_gbn(_ptr(part6), B, C, V, int(n_total),
                                                  _ptr(dy_coef), _ptr(dy_st.mean),
                                                  _ptr(st.mean), _ptr(st.invstd),
                                                  _ptr(bn.weight), _ptr(dgamma), _ptr(dbeta), 0,
                                                  int(st.batch), _ptr(coef), _stream(part6))
    _lib.check(rc, "sgcn_bn_bwd_finalize_gbn")
    return coef, dgamma, dbeta


def bn_bwd_apply(dy, y, relu, x, coef, per_joint, r=None, rcoef=None, dr=None, dx=None,
                 dy_coef=None):
    B, C, T, V = x.shape
    dx = torch.empty_like(x) if dx is None else dx
    nb = 4 * x.numel() * (3 + (y is not None) + (r is not None) + (dr is not None))
    with _timed("bn_bwd_apply", 0, nb, x, _shp(x)):
        rc = _lib.load().sgcn_bn_bwd_apply(
            _ptr(dy), _ptr(y), int(relu), _ptr(x), _ptr(coef), int(per_joint), _ptr(r),
            _ptr(rcoef), _ptr(dy_coef), _ptr(dx), _ptr(dr), B, C, T, V, _stream(x))
    _lib.check(rc, "sgcn_bn_bwd_apply")
    return dx


def mask_prep(mask):
    check_input(mask, "Feature_Mask")
    m = torch.empty_like(mask)
    with _timed("finalize", 0, 8 * mask.numel(), mask):
        rc = _lib.load().sgcn_mask_prep(_ptr(mask), _ptr(m), mask.numel(), _stream(mask))
    _lib.check(rc, "sgcn_mask_prep")
    return m


def _arr(ctype, vals):
    return (ctype * len(vals))(*vals)


def _chunks(xs):
    for i in range(0, len(xs), _lib.BATCH_MAX):
        yield xs[i:i + _lib.BATCH_MAX]


def mask_prep_many(masks):
    """tanh(mask) + 1 of several Feature_Masks in ONE launch per SGCN_BATCH_MAX
    (sgcn_mask_prep_many; the entries are kernel arguments, nothing is copied)."""
    outs = []
    for ch in _chunks(list(masks)):
        for mk in ch:
            check_input(mk, "Feature_Mask")
        o = [torch.empty_like(mk) for mk in ch]
        with _timed("finalize", 0, 8 * sum(m.numel() for m in ch), ch[0]):
            rc = _lib.load().sgcn_mask_prep_many(
                _arr(ctypes.c_void_p, [m.data_ptr() for m in ch]),
                _arr(ctypes.c_void_p, [t.data_ptr() for t in o]),
                _arr(ctypes.c_int, [m.numel() for m in ch]), len(ch), _stream(ch[0]))
        _lib.check(rc, "sgcn_mask_prep_many")
        outs += o
    return outs


def pos_finalize_many(entries):
    """Several deferred position-gradient finalizes [(PosPartials, gx, gy)] in one launch
    per SGCN_BATCH_MAX (sgcn_tshift_pos_finalize_many), on the current stream."""
    for ch in _chunks(list(entries)):
        for _, gx, gy in ch:
            check_input(gx, "gx")
            check_input(gy, "gy")
        with _timed("finalize", 0, sum(pp.ws.numel() * 4 for pp, _, _ in ch), ch[0][1]):
            rc = _lib.load().sgcn_tshift_pos_finalize_many(
                _arr(ctypes.c_void_p, [pp.ws.data_ptr() for pp, _, _ in ch]),
                _arr(ctypes.c_void_p, [gx.data_ptr() for _, gx, _ in ch]),
                _arr(ctypes.c_void_p, [gy.data_ptr() for _, _, gy in ch]),
                _arr(ctypes.c_int, [pp.B for pp, _, _ in ch]),
                _arr(ctypes.c_int, [pp.C for pp, _, _ in ch]), len(ch), _stream(ch[0][1]))
        _lib.check(rc, "sgcn_tshift_pos_finalize_many")


def mask_grad_finalize_many(entries):
    """Several deferred mask-gradient finalizes [(part, mask, B, C, V, dmask)] in one launch
    per SGCN_BATCH_MAX (sgcn_mask_grad_finalize_many), on the current stream."""
    for ch in _chunks(list(entries)):
        for e in ch:
            check_input(e[5], "dmask")
        with _timed("finalize", 0, sum(e[0].numel() * 4 for e in ch), ch[0][0]):
            rc = _lib.load().sgcn_mask_grad_finalize_many(
                _arr(ctypes.c_void_p, [e[0].data_ptr() for e in ch]),
                _arr(ctypes.c_void_p, [e[1].data_ptr() for e in ch]),
                _arr(ctypes.c_void_p, [e[5].data_ptr() for e in ch]),
                _arr(ctypes.c_int, [e[2] for e in ch]), _arr(ctypes.c_int, [e[3] for e in ch]),
                _arr(ctypes.c_int, [e[4] for e in ch]), len(ch), _stream(ch[0][0]))
        _lib.check(rc, "sgcn_mask_grad_finalize_many")


def gcn_gather(x0, m):
    B, C, T, V = x0.shape
    xg = torch.empty_like(x0)
    with _timed("gcn_gather", 0, 8 * x0.numel(), x0, _shp(x0)):
        rc = _lib.load().sgcn_gcn_gather(_ptr(x0), _ptr(m), _ptr(xg), B, C, T, V,
                                         _stream(x0))
    _lib.check(rc, "sgcn_gcn_gather")
    return xg


def gcn_dx_finish(dxt, x0, m, add1=None, add2=None, prev=None, add2_mask=None):
    """Returns (dx, dmask partials[, prev_part]); ``prev`` = (S, BnStats) of the previous
    unit's bn2 adds its backward-reduce partials (see sgcn_gcn_dx_finish)."""
    B, C, T, V = dxt.shape
    dx = torch.empty_like(dxt)
    part = torch.empty((B * C * V,), device=dxt.device, dtype=_F32)
    pp = torch.empty((B * C * 2,), device=dxt.device, dtype=_F32) if prev is not None else None
    ps, pst = prev if prev is not None else (None, None)
    nb = 4 * dxt.numel() * (3 + sum(t is not None for t in (add1, add2, add2_mask, ps)))
    with _timed("gcn_dx_finish", 0, nb, dxt, _shp(dxt)):
        rc = _lib.load().sgcn_gcn_dx_finish(_ptr(dxt), _ptr(x0), _ptr(m), _ptr(add1),
                                            _ptr(add2), _ptr(add2_mask), _ptr(dx), _ptr(part),
                                            _ptr(ps), _ptr(pst.mean) if pst else None,
                                            _ptr(pst.invstd) if pst else None, _ptr(pp), B, C,
                                            T, V, _stream(dxt))
    _lib.check(rc, "sgcn_gcn_dx_finish")
    return (dx, part) if prev is None else (dx, part, pp)


def mask_grad_finalize(part, mask, B, C, V, out=None):
    dmask = torch.empty_like(mask) if out is None else out
    with _timed("finalize", 0, 4 * part.numel(), mask):
        rc = _lib.load().sgcn_mask_grad_finalize(_ptr(part), _ptr(mask), B, C, V, _ptr(dmask),
                                                 0, _stream(mask))
    _lib.check(rc, "sgcn_mask_grad_finalize")
    return dmask


# --------------------------------------------------------------------------------------
# model head (permute + data_bn) and tail (global average pool), shift_gcn.py:193-216
# --------------------------------------------------------------------------------------
def head_moments(x):
    """{mean, M2} over t per (n, data_bn feature) of the (N, C, T, V, M) clip."""
    check_input(x, "input")
    N, C, T, V, M = x.shape
    part = torch.empty((N * M * V * C * 2,), device=x.device, dtype=_F32)
    with _timed("head", 0, 4 * x.numel(), x):
        rc = _lib.load().sgcn_head_moments(_ptr(x), _ptr(part), N, C, T, V, M, _stream(x))
    _lib.check(rc, "sgcn_head_moments")
    return part


def head_apply(x, st: BnStats):
    """Planes (N*M, C, T, V) = data_bn(permuted clip) with the coefficients of ``st``."""
    N, C, T, V, M = x.shape
    y = torch.empty((N * M, C, T, V), device=x.device, dtype=_F32)
    with _timed("head", 0, 8 * x.numel(), x):
        rc = _lib.load().sgcn_head_apply(_ptr(x), _ptr(st.scale), _ptr(st.shift), _ptr(y), N, C,
                                         T, V, M, _stream(x))
    _lib.check(rc, "sgcn_head_apply")
    return y


def head_bwd_reduce(g, x, st: BnStats):
    check_input(g, "grad_output")
    N, C, T, V, M = x.shape
    part = torch.empty((N * M * V * C * 2,), device=x.device, dtype=_F32)
    with _timed("head", 0, 8 * x.numel(), x):
        rc = _lib.load().sgcn_head_bwd_reduce(_ptr(g), _ptr(x), _ptr(st.mean), _ptr(st.invstd),
                                              _ptr(part), N, C, T, V, M, _stream(x))
    _lib.check(rc, "sgcn_head_bwd_reduce")
    return part


def head_bwd_apply(g, x, coef):
    N, C, T, V, M = x.shape
    dx = torch.empty_like(x)
    with _timed("head", 0, 12 * x.numel(), x):
        rc = _lib.load().sgcn_head_bwd_apply(_ptr(g), _ptr(x), _ptr(coef), _ptr(dx), N, C, T, V,
                                             M, _stream(x))
    _lib.check(rc, "sgcn_head_bwd_apply")
    return dx


def pool(x, N, M):
    """(N*M, C, T, V) -> (N, C): x.view(N, M, C, -1).mean(3).mean(1)."""
    check_input(x, "input")
    C = x.shape[1]
    P = x.numel() // max(1, N * M * C)
    out = torch.empty((N, C), device=x.device, dtype=_F32)
    with _timed("pool", 0, 4 * x.numel(), x):
        rc = _lib.load().sgcn_pool(_ptr(x), _ptr(out), N, M, C, P, _stream(x))
    _lib.check(rc, "sgcn_pool")
    return out


def pool_bwd(dout, shape, N, M):
    check_input(dout, "grad_output")
    dx = torch.empty(shape, device=dout.device, dtype=_F32)
    C = shape[1]
    P = dx.numel() // max(1, N * M * C)
    with _timed("pool", 0, 4 * dx.numel(), dout):
        rc = _lib.load().sgcn_pool_bwd(_ptr(dout), _ptr(dx), N, M, C, P, _stream(dout))
    _lib.check(rc, "sgcn_pool_bwd")
    return dx
