"""Fused forward/backward recipes of the Shift-GCN blocks on the HIP library.

Each block of ``model/shift_gcn.py`` is computed by a short, fixed sequence of C-ABI
launches (no torch compute ops), with its backward written out explicitly so that the
fusions survive training:

Shift_gcn (shift_gcn.py:121-142)
  fwd : gather[shift_in * mask, written by the previous unit's tail launch]
        -> pw_fwd[einsum + bias; Z stored before shift_out]
        -> moments(per joint, shift_out in the addressing) -> bn_finalize
        -> [down: pw_fwd -> moments -> finalize] -> bn_apply(+down/identity, ReLU)
  bwd : per-joint BN partials (from the Shift_tcn shift_in backward, or bn_bwd_reduce)
        -> finalize -> bn_bwd_apply[dZ in Z's layout] -> pw_fwd(dX) -> pw_dw(Linear_weight^T,
        bias) -> gcn_dx_finish(shift_in^T + mask, dmask partials) -> mask_grad_finalize
        -> [down: pw_fwd(accumulate), pw_dw]
Shift_tcn (shift_gcn.py:65-74)
  fwd : finalize(bn) -> tshift_fwd[bn affine fused on taps] -> pw_fwd[temporal_linear +
        bias + ReLU] (C = 256: both in one pw_fwd_tshift) -> tshift_fwd[stride s, bn2
        moments fused] -> finalize(bn2) -> (standalone: bn_apply)
  bwd : tshift_bwd[ReLU mask fused; in a unit also bn2's input gradient] -> pw_fwd(dX)
        -> pw_dw -> tshift_bwd[bn affine + bn-backward partials fused] -> finalize
        -> (standalone: bn_bwd_apply; in a unit the BN input gradient is never written: the
           gcn BN-backward kernels evaluate it on the fly)
TCN_GCN_unit (shift_gcn.py:160-162): bn2 apply + residual (0 / identity / tcn conv+BN) +
  ReLU is ONE bn_apply launch; its backward ONE reduce + ONE apply.

Everything runs on torch's current stream; intermediate buffers come from torch's
caching allocator, so a whole training step can be captured in a hipGraph.
"""
from __future__ import annotations

import os
import threading

import torch

from . import ops
from .ops import PlaneView as PV


def _empty(*shape, like):
    return torch.empty(shape, device=like.device, dtype=torch.float32)


# --------------------------------------------------------------------------------------
# Off-critical-path launches (weight gradients). In a linked chain of units (Model.forward)
# the weight/bias gradients of every contraction are needed only by the optimizer, so their
# contractions (MFMA-bound split-K GEMMs + slab reductions) are enqueued on a SIDE stream and
# run concurrently with the HBM-bound streaming kernels of the input-gradient chain. The
# first unit of the chain (whose backward runs last) joins the side stream back into the
# current stream before returning, so everything after loss.backward() sees finished grads.
# --------------------------------------------------------------------------------------
_SIDE = {}


def _side_stream(device):
    s = _SIDE.get(device)
    if s is None:
        s = _SIDE[device] = torch.cuda.Stream(device=device)
    return s


class _OffPath:
    """``with _OffPath(on, *operands):`` enqueue the enclosed launches on the side stream,
    after everything already enqueued on the current stream. Outputs must be allocated
    BEFORE entering (current-stream memory, joined later); the operands read on the side
    stream are marked with ``record_stream`` so the caching allocator does not hand their
    memory to the current stream while the side stream may still read it."""

    __slots__ = ("on", "tensors", "side", "ctx", "ev")

    def __init__(self, on, *tensors):
        self.on = bool(on)
        self.tensors = tensors

    def __enter__(self):
        if not self.on:
            return self
        dev = self.tensors[0].device
        main = torch.cuda.current_stream(dev)
        self.side = _side_stream(dev)
        self.side.wait_stream(main)
        self.ctx = torch.cuda.stream(self.side)
        self.ctx.__enter__()
        return self

    def __exit__(self, *exc):
        if not self.on:
            return False
        self.ctx.__exit__(*exc)
        for t in self.tensors:
            if t is not None:
                t.record_stream(self.side)
        self.ev = torch.cuda.Event()
        self.ev.record(self.side)
        return False

    def wait(self):
        """Make the current stream wait for the enclosed launches (no-op when off)."""
        if self.on:
            torch.cuda.current_stream(self.tensors[0].device).wait_event(self.ev)


# --------------------------------------------------------------------------------------
# Deferred gradient writes. A gradient written AFTER its block's backward has returned (a
# weight gradient on the side stream, an optimizer-only finalize batched to the end of the
# backward) is never handed to autograd: the block returns None for that parameter, and the
# end-of-backward callback (_finish), once the side stream is joined, accumulates the tensor
# into ``.grad`` itself, DDP-style. Autograd therefore never sums or copies an unwritten
# tensor, whatever else contributes to the parameter's gradient in the same backward (a
# regulariser in the loss, a parameter tied across blocks, the model used twice in one
# graph, an existing ``.grad``). A parameter whose gradient autograd must see during the
# backward (hooks, ``torch.autograd.grad`` capturing it, ``create_graph``) is not deferred.
# --------------------------------------------------------------------------------------
# Optimizer-only finalizes (position and mask gradients) are deferred to the end of the
# backward and launched together: one launch per kind instead of one per unit
# (SGCN_BATCH_SIDE=0: each its own launch, as before).
BATCH_SIDE = int(os.environ.get("SGCN_BATCH_SIDE", "1"))


class _Later:
    """A gradient tensor written after the block's backward returns (see above)."""

    __slots__ = ("t",)

    def __init__(self, t):
        self.t = t


def _late(t, off):
    return _Later(t) if off else t


class _Task:
    """One backward pass's deferred work on one device: position / mask finalizes,
    (parameter, gradient) pairs to accumulate, whether the side stream was used."""

    __slots__ = ("pos", "mask", "grads", "side")

    def __init__(self):
        self.pos, self.mask, self.grads, self.side = [], [], [], False


# (device, graph task id) -> _Task. A backward that raises never runs its callback, so its
# entry (and the tensors it holds) stays; it is not purged by id, because concurrent
# backwards from other threads share the device's worker thread and a later id may be live.
_TASKS = {}


def _task(device):
    """The current backward's _Task on ``device``; the first use queues its end-of-backward
    callback (the engine runs final callbacks on the caller's stream, after every node)."""
    key = (device, torch._C._current_graph_task_id())
    t = _TASKS.get(key)
    if t is None:
        t = _TASKS[key] = _Task()
        torch.autograd.Variable._execution_engine.queue_callback(lambda: _finish(key))
    return t


def _defer_ok(params):
    """Whether the gradients of ``params`` may be written after the block's backward
    returns: a plain backward that will run their AccumulateGrad (not
    ``torch.autograd.grad`` capturing them, not ``backward(inputs=...)`` without them, not
    ``create_graph``) and nothing that reads a gradient during the backward (tensor hooks,
    post-accumulate-grad hooks)."""
    if torch.is_grad_enabled():
        return False   # create_graph: AccumulateGrad differentiates through the sum
    for p in params:
        if (getattr(p, "_backward_hooks", None) or
                getattr(p, "_post_accumulate_grad_hooks", None)):
            return False
        try:
            if not torch._C._will_engine_execute_node(
                    torch.autograd.graph.get_gradient_edge(p).node):
                return False
        except RuntimeError:   # torch.autograd.grad returns p's gradient: not deferred
            return False
    return True


def _accumulate(p, g):
    """``.grad += g`` for a deferred gradient (AccumulateGrad's rule: take g when .grad is
    None, else add in place), keeping p's gradient-bucket slot as .grad when g is it."""
    cur = p.grad
    if cur is None:
        p.grad = g
    elif ops.is_grad_slot(p, g) and not ops.is_grad_slot(p, cur):
        g.add_(cur)        # (a + b == b + a bit for bit)
        p.grad = g
    else:
        cur.add_(g)


def _finish(key):
    """End of a backward: the deferred finalizes (on the current stream before its wait
    for the side stream, TAIL_MAIN bit 1, else on the side stream), the wait, then every
    deferred gradient accumulated into its parameter's .grad."""
    t = _TASKS.pop(key, None)
    if t is None:
        return
    dev = key[0]
    if t.pos or t.mask:
        keep = [e[0].ws for e in t.pos] + [e[0] for e in t.mask]
        with _OffPath(t.side and not (TAIL_MAIN & 1), *keep):
            ops.pos_finalize_many(t.pos)
            ops.mask_grad_finalize_many(t.mask)
    s = _SIDE.get(dev)
    if t.side and s is not None:
        torch.cuda.current_stream(dev).wait_stream(s)
    for p, g in t.grads:
        _accumulate(p, g)


def _pos_grads(gx, gy, shift):
    """A shift backward's (grad_xpos, grad_ypos): as returned, or, when its partials were
    left for later (ops.PosPartials, a unit on the side stream), finalized after the
    backward into gradient tensors allocated here (batched with the backward's others when
    BATCH_SIDE) and handed over as deferred gradients."""
    if not isinstance(gx, ops.PosPartials):
        return gx, gy
    ox, oy = ops.grad_like(shift.xpos), ops.grad_like(shift.ypos)
    if BATCH_SIDE:
        _task(gx.ws.device).pos.append((gx, ox, oy))
    else:
        with _OffPath(True, gx.ws):
            gx.finalize(ox, oy)
    return _Later(ox), _Later(oy)


def _pos_alloc(shift, off):
    """Gradient tensors for a shift backward's (xpos, ypos) gradients (their bucket slots
    when registered, ops.grad_like), or None when they are deferred to the side stream."""
    return None if off else (ops.grad_like(shift.xpos), ops.grad_like(shift.ypos))


# End of the backward (A/B knob SGCN_TAIL_MAIN, bits): 1 = the deferred finalizes launch on
# the current stream BEFORE its wait for the side stream (the wait then finds the side's
# last weight gradients done or nearly so); 2 = the chain's first unit (the last backward)
# keeps its weight gradients on the current stream (linked_units)
TAIL_MAIN = int(os.environ.get("SGCN_TAIL_MAIN", "3"))


# ======================================================================================
# Shift_gcn
# ======================================================================================
class GcnSaved:
    __slots__ = ("x0", "xg", "Z", "zst", "D0", "dst", "H", "m", "h_moments")


def gcn_forward(mod, x0, training, off=False):
    """``off``: the down conv branch (contraction + statistics) runs on the side stream,
    concurrently with the gcn contraction, joined before the apply that reads it."""
    B, Cin, T, V = x0.shape
    Cout = mod.out_channels
    D0 = dst = None
    if mod.has_down:
        conv, bn = mod.down[0], mod.down[1]
        D0 = _empty(B, Cout, T, V, like=x0)
        down = _OffPath(off, x0)
        with down:
            ops.pw_fwd(conv.weight, False, conv.bias, PV(x0), PV(D0), Cout, Cin, T, V)
            if training:
                dst = ops.bn_finalize(ops.moments(D0, False), B, Cout, T * V, bn)
            else:
                dst = ops.bn_eval_coef(bn, Cout)
    cache = mod.__dict__.pop("_gather_cache", None)
    if cache is not None and cache[0] is x0:
        xg, m = cache[1], cache[2]    # made by the previous unit's tail from its registers
    else:
        m = _mask_of(mod)
        xg = ops.gcn_gather(x0, m)    # shift_in gather * mask, once (reused by the dW)
    Z = _empty(B, Cout, T, V, like=x0)
    # Z is stored BEFORE shift_out (plain contraction stores) and the BatchNorm kernels
    # apply the joint rotation in their addressing (per_joint = 3)
    ops.pw_fwd(mod.Linear_weight, True, mod.Linear_bias, PV(xg), PV(Z), Cout, Cin, T, V)
    if training:
        zst = ops.bn_finalize(ops.moments(Z, 3), B, Cout * V, T, mod.bn, perm_V=V)
    else:
        zst = ops.bn_eval_coef(mod.bn, Cout * V, perm_V=V)
    if mod.has_down:
        down.wait()
        H, hm = ops.bn_apply(Z, zst, 3, r=D0, rst=dst, relu=True, out_stats=training)
    else:
        H, hm = ops.bn_apply(Z, zst, 3, r=x0, relu=True, out_stats=training)
    s = GcnSaved()
    s.x0, s.xg, s.Z, s.zst, s.D0, s.dst, s.H, s.m = x0, xg, Z, zst, D0, dst, H, m
    s.h_moments = hm   # moments of H for Shift_tcn.bn, produced by the same launch
    return H, s


def _mask_of(gcn):
    """tanh(Feature_Mask) + 1 of a Shift_gcn: the one linked_units prepared for this call
    (all units' in one launch), else its own launch (once per version of the mask)."""
    fm = gcn.Feature_Mask
    r = gcn.__dict__.get("_mask_ready")
    if r is not None and r[0] is fm and r[1] == fm._version:
        return r[2]
    if gcn.training:
        return ops.mask_prep(fm)
    return ops.cached(gcn, "_sgcn_mask", ops._src_key((fm,)), lambda: ops.mask_prep(fm),
                      fm.device)


def prepare_masks(gcns):
    """Every Shift_gcn's mask for one forward in one launch (sgcn_mask_prep_many); in eval
    mode once per version of the masks (ops.cached)."""
    fms = [g.Feature_Mask for g in gcns]
    if any(g.training for g in gcns):
        ms = ops.mask_prep_many(fms)
    else:
        ms = ops.cached(gcns[0], "_sgcn_masks", ops._src_key(fms) + tuple(map(id, gcns)),
                        lambda: ops.mask_prep_many(fms), fms[0].device)
    for g, m in zip(gcns, ms):
        g.__dict__["_mask_ready"] = (g.Feature_Mask, g.Feature_Mask._version, m)


def gcn_backward(mod, s: GcnSaved, dH, extra_dx=None, dy_coef=None, prev=None, extra_out=None,
                 pre6=None, off=False):
    """Returns (dx0, {param_name: grad}). With ``dy_coef`` ([3, Cout]) the incoming
    gradient is dH = k1*dH_arg + k2*H + k3 (Shift_tcn.bn's input gradient), evaluated
    on the fly by the BN-backward kernels instead of being materialised. ``pre6`` =
    (six-sum partials, Shift_tcn.bn stats) from sgcn_tshift_bwd_gbn: bn's backward
    partials were made by the shift_in backward launch (no reduce pass here). ``off``:
    the weight-gradient launches go to the side stream (see _OffPath)."""
    x0 = s.x0
    B, Cin, T, V = x0.shape
    Cout = mod.out_channels
    g = {}
    rpart = None
    if pre6 is not None:
        assert dy_coef is not None and (pre6[2] is not None) == mod.has_down
        coefZ, g["bn.weight"], g["bn.bias"] = ops.bn_bwd_finalize_gbn(
            pre6[0], B, Cout, V, B * T, dy_coef, pre6[1], s.zst, mod.bn)
    else:
        if mod.has_down:
            conv, bnd = mod.down[0], mod.down[1]
            part, rpart = ops.bn_bwd_reduce(dH, s.H, True, s.Z, s.zst, 3, r=s.D0,
                                            rst=s.dst, dy_coef=dy_coef)
        else:
            part, rpart = ops.bn_bwd_reduce(dH, s.H, True, s.Z, s.zst, 3, dy_coef=dy_coef)
        coefZ, g["bn.weight"], g["bn.bias"] = ops.bn_bwd_finalize(part, B, Cout * V, B * T,
                                                                   s.zst, mod.bn, perm_V=V)
    dZ = _empty(B, Cout, T, V, like=x0)
    g_id = dD0 = None
    if mod.has_down:
        conv, bnd = mod.down[0], mod.down[1]
        if pre6 is not None:   # the down BatchNorm's six plane sums, from the same launch
            coefD, g["down.1.weight"], g["down.1.bias"] = ops.bn_bwd_finalize_gbn(
                pre6[2], B, Cout, 1, B * T * V, dy_coef, pre6[1], s.dst, bnd)
        else:
            coefD, g["down.1.weight"], g["down.1.bias"] = ops.bn_bwd_finalize(
                rpart, B, Cout, B * T * V, s.dst, bnd)
        dD0 = _empty(B, Cout, T, V, like=x0)
        ops.bn_bwd_apply(dH, s.H, True, s.Z, coefZ, 3, r=s.D0, rcoef=coefD, dr=dD0, dx=dZ,
                         dy_coef=dy_coef)
    else:
        g_id = _empty(B, Cin, T, V, like=x0)
        ops.bn_bwd_apply(dH, s.H, True, s.Z, coefZ, 3, dr=g_id, dx=dZ, dy_coef=dy_coef)
    # dZ is stored in Z's pre-shift_out layout, so the einsum/bias grads and dX read it as
    # a plain plane: G(b,d,n) = dZ[b,d,n]
    dLW = ops.grad_like(mod.Linear_weight)
    dLb = ops.grad_like(mod.Linear_bias)
    dXt = _empty(B, Cin, T, V, like=x0)
    # on the side stream the weight gradient is enqueued after the dX contraction (it then
    # overlaps the streaming passes that follow instead of competing for the MFMA pipes)
    ops.pw_fwd(mod.Linear_weight, False, None, PV(dZ), PV(dXt), Cin, Cout, T, V)
    with _OffPath(off, dZ, s.xg):
        ops.pw_dw(PV(dZ), PV(s.xg), dLW, Cout, Cin, T, V, transpose=True, dbias=dLb)
    g["Linear_weight"], g["Linear_bias"] = _late(dLW, off), _late(dLb, off)
    a2, a2m = extra_dx if isinstance(extra_dx, tuple) else (extra_dx, None)
    if prev is not None:   # also the previous unit's bn2 backward partials (x0 = its out)
        dx, mpart, extra_out["prev_part"] = ops.gcn_dx_finish(dXt, x0, s.m, add1=g_id,
                                                              add2=a2, prev=prev,
                                                              add2_mask=a2m)
    else:
        dx, mpart = ops.gcn_dx_finish(dXt, x0, s.m, add1=g_id, add2=a2, add2_mask=a2m)
    dmask = ops.grad_like(mod.Feature_Mask)
    fm = mod.Feature_Mask
    if BATCH_SIDE and (off or _defer_ok((fm,))):
        # with the backward's other optimizer-only finalizes (end of the backward)
        _task(mpart.device).mask.append((mpart, fm, B, Cin, V, dmask))
        g["Feature_Mask"] = _Later(dmask)
    else:
        with _OffPath(off, mpart):
            ops.mask_grad_finalize(mpart, fm, B, Cin, V, out=dmask)
        g["Feature_Mask"] = _late(dmask, off)
    if mod.has_down:
        dWd = ops.grad_like(conv.weight)
        dbd = ops.grad_like(conv.bias)
        ops.pw_fwd(conv.weight, True, None, PV(dD0), PV(dx), Cin, Cout, T, V, accumulate=True)
        with _OffPath(off, dD0, x0):
            ops.pw_dw(PV(dD0), PV(x0), dWd, Cout, Cin, T, V, dbias=dbd)
        g["down.0.weight"], g["down.0.bias"] = _late(dWd, off), _late(dbd, off)
    return dx, g


# ======================================================================================
# Shift_tcn
# ======================================================================================
class TcnSaved:
    __slots__ = ("H", "ast", "As", "R", "S", "sst")


def tshift_fused(C):
    """Whether Shift_tcn's shift_in is formed inside temporal_linear's operand staging
    (sgcn_pw_fwd_tshift) at C input channels: from TSHIFT_FUSION_MIN_C up."""
    return C >= TSHIFT_FUSION_MIN_C


def folded_conv_bn(conv, bn):
    """Eval-mode conv -> BatchNorm with nothing in between (``down`` = Conv2d + BN2d,
    shift_gcn.py:83-86; ``tcn`` = Conv2d + BN2d, :31-45) folded into ONE conv: weight
    ``W * s[o]``, bias ``b * s + t`` with the BatchNorm's eval apply coefficients
    (s = gamma * invstd, t = beta - mean * s, sgcn_bn_eval_coef). Computed once and cached
    on the conv, keyed by the storage and version counters of every tensor it reads, so an
    optimizer step, load_state_dict or a device move recomputes it."""
    srcs = (conv.weight, conv.bias, bn.weight, bn.bias, bn.running_mean, bn.running_var)
    key = ops._src_key(srcs) + (float(bn.eps),)

    def make():
        st = ops.bn_eval_coef(bn, conv.out_channels)
        with torch.no_grad():
            w = (conv.weight.detach() *
                 st.scale.view(-1, *([1] * (conv.weight.dim() - 1)))).contiguous()
            b = (conv.bias.detach() * st.scale + st.shift if conv.bias is not None
                 else st.shift.clone())
        return w, b
    return ops.cached(conv, "_sgcn_fold", key, make, conv.weight.device)


def convbn_infer_folded(mod, x):
    """Inference residual ``tcn`` (kernel 1, stride s): the conv with its BatchNorm
    folded in, one contraction; returns its output (no affine left for the consumer)."""
    B, Cin, T, V = x.shape
    conv = mod.conv
    Cout = conv.out_channels
    To = (T - 1) // mod.stride + 1
    w, b = folded_conv_bn(conv, mod.bn)
    R = _empty(B, Cout, To, V, like=x)
    ops.pw_fwd(w, False, b, PV(x, mod.stride), PV(R), Cout, Cin, To, V)
    return R


def gcn_infer_z(mod, x0):
    """Inference Shift_gcn up to its contraction output: (Z, zst, res, res_stats); the
    BN1d + down/identity + ReLU are applied by the consumer (sgcn_tshift_fwd_pre)."""
    B, Cin, T, V = x0.shape
    Cout = mod.out_channels
    cache = mod.__dict__.pop("_gather_cache", None)
    if cache is not None and cache[0] is x0:
        xg = cache[1]
    else:
        xg = ops.gcn_gather(x0, _mask_of(mod))
    Z = _empty(B, Cout, T, V, like=x0)
    ops.pw_fwd(mod.Linear_weight, True, mod.Linear_bias, PV(xg), PV(Z, 1, +1), Cout, Cin, T, V)
    zst = ops.bn_eval_coef(mod.bn, Cout * V, perm_V=V)
    if mod.has_down:
        conv, bn = mod.down[0], mod.down[1]
        D0 = _empty(B, Cout, T, V, like=x0)
        if EVAL_FOLD:   # down.1 folded into down.0: the residual needs no affine
            w, b = folded_conv_bn(conv, bn)
            ops.pw_fwd(w, False, b, PV(x0), PV(D0), Cout, Cin, T, V)
            return Z, zst, D0, None
        ops.pw_fwd(conv.weight, False, conv.bias, PV(x0), PV(D0), Cout, Cin, T, V)
        return Z, zst, D0, ops.bn_eval_coef(bn, Cout)
    return Z, zst, x0, None


def tcn_core_forward(mod, H, training, h_moments=None, tail=None, pre=None):
    """bn -> shift_in -> temporal_linear -> ReLU -> shift_out; returns (S, bn2 stats, saved)
    where S is the shift_out output BEFORE bn2. ``h_moments``: per-plane moments of H
    already produced by the launch that wrote H (else computed here)."""
    src = H if H is not None else pre[0]
    B, C, T, V = src.shape
    Cout = mod.out_channels
    si, so = mod.shift_in, mod.shift_out
    stride = so.stride
    if training:
        if h_moments is None:
            h_moments = ops.moments(H, False)
        ast = ops.bn_finalize(h_moments, B, C, T * V, mod.bn)
    else:
        ast = ops.bn_eval_coef(mod.bn, C)
    R = _empty(B, Cout, T, V, like=src)
    tl = mod.temporal_linear
    As = None
    if pre is not None:   # inference: H = relu(BN1d(Z) + res) formed while staging
        As = ops.tshift_fwd_pre(pre[0], si.xpos.detach(), si.ypos.detach(), si.stride, pre[1],
                                pre[2], pre[3], ast)
        ops.pw_fwd(tl.weight, False, tl.bias, PV(As), PV(R), Cout, C, T, V, relu=True)
    elif tshift_fused(C) and tail is None:
        # shift_in (with Shift_tcn.bn's apply) formed in the contraction's operand staging,
        # never read back; also stored from the same registers for the weight gradient
        As = torch.empty_like(H)
        ops.pw_fwd_tshift(tl.weight, tl.bias, PV(H), si.xpos.detach(), si.ypos.detach(), ast,
                          PV(R), Cout, C, T, V, relu=True, x_shifted=As, two_row=TSHIFT_TWO_ROW)
    else:
        As = ops.tshift_fwd(H, si.xpos.detach(), si.ypos.detach(), si.stride, affine=ast)
        ops.pw_fwd(tl.weight, False, tl.bias, PV(As), PV(R), Cout, C, T, V, relu=True)
    To = T // stride
    if tail is not None:
        # inference: bn2 (eval) + residual + ReLU (+ next gather) fused into shift_out
        sst = ops.bn_eval_coef(mod.bn2, Cout)
        return ops.tshift_fwd_tail(R, so.xpos.detach(), so.ypos.detach(), stride, sst,
                                   r=tail[0], rst=tail[1], gather_m=tail[2])
    stats = _empty(B * Cout * 2, like=src) if training else None
    S = ops.tshift_fwd(R, so.xpos.detach(), so.ypos.detach(), stride, stats=stats)
    if training:
        sst = ops.bn_finalize(stats, B, Cout, To * V, mod.bn2)
    else:
        sst = ops.bn_eval_coef(mod.bn2, Cout)
    s = TcnSaved()
    s.H, s.ast, s.As, s.R, s.S, s.sst = H, ast, As, R, S, sst
    return S, sst, s


def tcn_core_backward(mod, s: TcnSaved, dS, materialize_dx=True, gpre=None, gcn_z=None,
                      out=None, off=False):
    """dS: gradient w.r.t. S (pre-bn2). Returns (dH, grads), or ((dA, coef), grads) with
    ``materialize_dx=False`` (dH = coef[0]*dA + coef[1]*H + coef[2], fused downstream).
    ``gcn_z`` = (Z, zst[, (D0, dst)]) of the producing Shift_gcn: its BatchNorm's (and its
    down BatchNorm's) backward sums come out of the shift_in backward launch, returned as
    out["pre6"] = (z sums, Shift_tcn.bn stats, down sums or None)."""
    H = s.H
    B, C, T, V = H.shape
    Cout = mod.out_channels
    si, so = mod.shift_in, mod.shift_out
    g = {}
    # (off: each shift backward leaves its position-gradient partials for a finalize on the
    # side stream, _pos_grads: the positions' gradients only feed the optimizer)
    if gpre is not None:   # dS = bn2's input gradient, formed inside the shift backward
        dRp, gx, gy = ops.tshift_bwd_bnin(gpre[0], gpre[1], s.S, gpre[2], s.R,
                                          so.xpos.detach(), so.ypos.detach(), defer_pos=off,
                                          pos_out=_pos_alloc(so, off))
    else:
        dRp, gx, gy = ops.tshift_bwd(dS, s.R, so.xpos.detach(), so.ypos.detach(), so.stride,
                                     relu_mask=True, defer_pos=off,
                                     pos_out=_pos_alloc(so, off))
    g["shift_out.xpos"], g["shift_out.ypos"] = _pos_grads(gx, gy, so)
    tl = mod.temporal_linear
    dWt = ops.grad_like(tl.weight)
    dbt = ops.grad_like(tl.bias)

    dAs = _empty(B, C, T, V, like=H)
    ops.pw_fwd(tl.weight, True, None, PV(dRp), PV(dAs), C, Cout, T, V)
    with _OffPath(off, dRp, s.As):   # after the dX contraction (see gcn_backward)
        ops.pw_dw(PV(dRp), PV(s.As), dWt, Cout, C, T, V, dbias=dbt)
    g["temporal_linear.weight"], g["temporal_linear.bias"] = _late(dWt, off), _late(dbt, off)
    # shift_in backward with Shift_tcn.bn's backward partials fused in (and, GBN, those of
    # the Shift_gcn BatchNorm that produced H)
    if gcn_z is not None and GBN_FUSION and si.stride == 1 and ops.ra_fits(T * V, V):
        down = gcn_z[2] if len(gcn_z) > 2 else None
        res = ops.tshift_bwd_gbn(dAs, H, si.xpos.detach(), si.ypos.detach(), s.ast, gcn_z[0],
                                 gcn_z[1], defer_pos=off, down=down,
                                 pos_out=_pos_alloc(si, off))
        dA, gx, gy, part, zpart = res[:5]
        out["pre6"] = (zpart, s.ast, res[5] if down is not None else None)
    else:
        dA, gx, gy, part = ops.tshift_bwd(
            dAs, H, si.xpos.detach(), si.ypos.detach(), si.stride, scale=s.ast.scale,
            shift=s.ast.shift, bn_stats=s.ast, defer_pos=off, pos_out=_pos_alloc(si, off))
    g["shift_in.xpos"], g["shift_in.ypos"] = _pos_grads(gx, gy, si)
    coef, g["bn.weight"], g["bn.bias"] = ops.bn_bwd_finalize(part, B, C, B * T * V, s.ast,
                                                             mod.bn)
    if not materialize_dx:
        return (dA, coef), g       # dH = k1*dA + k2*H + k3, left for the consumer to fuse
    dH = ops.bn_bwd_apply(dA, None, False, H, coef, False)
    return dH, g


# ======================================================================================
# tcn (kernel_size = 1 residual conv + BN)
# ======================================================================================
class ConvBnSaved:
    __slots__ = ("x", "Rc", "rst", "To")


def convbn_core_forward(mod, x, training):
    B, Cin, T, V = x.shape
    conv, bn = mod.conv, mod.bn
    Cout = conv.out_channels
    s_t = mod.stride
    To = (T - 1) // s_t + 1
    Rc = _empty(B, Cout, To, V, like=x)
    ops.pw_fwd(conv.weight, False, conv.bias, PV(x, s_t), PV(Rc), Cout, Cin, To, V)
    if training:
        rst = ops.bn_finalize(ops.moments(Rc, False), B, Cout, To * V, bn)
    else:
        rst = ops.bn_eval_coef(bn, Cout)
    s = ConvBnSaved()
    s.x, s.Rc, s.rst, s.To = x, Rc, rst, To
    return Rc, rst, s


def convbn_dx_and_dw(mod, s: ConvBnSaved, dRc, dx, accumulate, off=False):
    """Conv weight/bias grads and dx (+)= W^T dRc at the strided rows."""
    B, Cin, T, V = s.x.shape
    conv = mod.conv
    Cout = conv.out_channels
    dW = ops.grad_like(conv.weight)
    db = ops.grad_like(conv.bias)
    ops.pw_fwd(conv.weight, True, None, PV(dRc), PV(dx, mod.stride), Cin, Cout, s.To, V,
               accumulate=accumulate)
    with _OffPath(off, dRc, s.x):
        ops.pw_dw(PV(dRc), PV(s.x, mod.stride), dW, Cout, Cin, s.To, V, dbias=db)
    return {"conv.weight": _late(dW, off), "conv.bias": _late(db, off)}


# ======================================================================================
# TCN_GCN_unit
# ======================================================================================
class UnitSaved:
    __slots__ = ("x", "gs", "ts", "rs", "out", "prev", "off")


def unit_forward(unit, x, training):
    consumer = unit.__dict__.get("_gather_consumer")
    if (not training and _INFER.active and
            x.shape[2] * x.shape[3] <= ops.TAIL_MAX_PLANE):
        # inference (no backward can follow): the Shift_gcn tail is fused into shift_in,
        # the unit tail into shift_out; neither H nor S is written
        # the Shift_gcn tail (BN1d eval + down/identity + ReLU) is formed in the shift_in
        # launch's staging
        pre = gcn_infer_z(unit.gcn1, x)
        r = rst = None
        if unit.residual_kind == "conv":
            if EVAL_FOLD:
                r = convbn_infer_folded(unit.residual, x)
            else:
                r, rst, _ = convbn_core_forward(unit.residual, x, training)
        elif unit.residual_kind == "identity":
            r = x
        gm = _mask_of(consumer) if consumer is not None else None
        out, xg_next = tcn_core_forward(unit.tcn1, None, training, tail=(r, rst, gm),
                                        pre=pre)
        if gm is not None:
            consumer.__dict__["_gather_cache"] = (out, xg_next, gm)
        return out, None
    # the previous unit's tail (its out is x): its bn2 backward partials are made by this
    # unit's gcn_dx_finish, which reads x anyway (see unit_backward); prev = (bn2 input
    # operand for ops.gcn_dx_finish, that unit)
    prev = unit.__dict__.pop("_prev_tail", None)
    prev = prev[1:] if prev is not None and prev[0] is x else None
    # linked chains only; not while a hipGraph is being captured (the graph replays one
    # stream's launches in order)
    off = (ASYNC_DW and bool(unit.__dict__.get("_off_path")) and
           not torch.cuda.is_current_stream_capturing())
    # the next unit's gcn mask (tanh(Feature_Mask) + 1), needed by this unit's tail launch:
    # a tiny kernel, made on the side stream off the critical path
    mp = None
    if consumer is not None:
        if "_mask_ready" in consumer.__dict__:   # prepared with the chain's others
            gm = _mask_of(consumer)
        else:
            mp = _OffPath(off, consumer.Feature_Mask)
            with mp:
                gm = ops.mask_prep(consumer.Feature_Mask)
    H, gs = gcn_forward(unit.gcn1, x, training, off=off)
    rs = None
    if unit.residual_kind == "conv":
        # the residual conv branch runs on the side stream, concurrently with Shift_tcn
        res = _OffPath(off, x)
        with res:
            Rc, rst, rs = convbn_core_forward(unit.residual, x, training)
    S, sst, ts = tcn_core_forward(unit.tcn1, H, training, h_moments=gs.h_moments)
    # the next unit's Shift_gcn (set by Model.forward_planes for the duration of a call):
    # its gathered, masked input is written by this tail launch too
    if mp is not None:
        mp.wait()
    elif consumer is None:
        gm = None
    if unit.residual_kind == "conv":
        res.wait()
        out = ops.bn_apply(S, sst, False, r=Rc, rst=rst, relu=True, gather_m=gm)
    elif unit.residual_kind == "identity":
        out = ops.bn_apply(S, sst, False, r=x, relu=True, gather_m=gm)
    else:
        out = ops.bn_apply(S, sst, False, relu=True, gather_m=gm)
    if gm is not None:
        out, xg_next = out
        consumer.__dict__["_gather_cache"] = (out, xg_next, gm)
    nxt = unit.__dict__.get("_next_unit")
    # the next unit's gcn_dx_finish may produce this unit's bn2 backward partials only if
    # the dx it reads is this unit's COMPLETE output gradient: no residual conv (whose dx is
    # added after) and no gcn down conv (whose dx is accumulated after gcn_dx_finish)
    if (nxt is not None and unit.residual_kind != "conv" and nxt.residual_kind != "conv"
            and not nxt.gcn1.has_down):
        nxt.__dict__["_prev_tail"] = (out, (S, sst), unit)
    s = UnitSaved()
    s.x, s.gs, s.ts, s.rs, s.out, s.prev = x, gs, ts, rs, out, prev
    s.off = off
    return out, s


def _gcn_z(unit, s: UnitSaved):
    """(Z, zst[, (D0, dst)]) of the unit's Shift_gcn: its BatchNorm's backward sums (and,
    with a down conv, the down BatchNorm's) come out of the shift_in backward launch."""
    # (sgcn_tshift_bwd_gbn reads Z in the pre-shift_out layout, D0 in the natural one)
    if unit.gcn1.has_down:
        return (s.gs.Z, s.gs.zst, (s.gs.D0, s.gs.dst)) if GBN_FUSION >= 2 else None
    return (s.gs.Z, s.gs.zst)


def _off_path_ok(unit, s: UnitSaved):
    """Weight gradients (and position / mask finalizes) of a linked unit may run on the side
    stream if every gradient of the unit may be deferred (_defer_ok): they are then handed
    to .grad at the end of the backward, after the join."""
    if not s.off or torch.cuda.is_current_stream_capturing():
        return False
    if not _defer_ok([p for p in unit.parameters() if p.requires_grad]):
        return False
    _task(s.x.device).side = True
    return True


def unit_backward(unit, s: UnitSaved, dout):
    return _unit_backward(unit, s, dout, _off_path_ok(unit, s))


def _unit_backward(unit, s: UnitSaved, dout, off):
    ts = s.ts
    S = ts.S
    so = unit.tcn1.shift_out
    B, Cout, To, V = S.shape
    kind = unit.residual_kind
    g = {}
    cached = unit.__dict__.pop("_bwd_part", None)
    if cached is not None and cached[0] is dout and kind != "conv":
        part, rpart = cached[1], None   # made by the next unit's gcn_dx_finish
    elif kind == "conv":
        part, rpart = ops.bn_bwd_reduce(dout, s.out, True, S, ts.sst, False, r=s.rs.Rc,
                                        rst=s.rs.rst)
    else:
        part, rpart = ops.bn_bwd_reduce(dout, s.out, True, S, ts.sst, False)
    coef2, g["tcn1.bn2.weight"], g["tcn1.bn2.bias"] = ops.bn_bwd_finalize(
        part, B, Cout, B * To * V, ts.sst, unit.tcn1.bn2)
    if kind != "conv" and so.stride == 1 and ops.ra_fits(To * V, V):
        # neither dS nor the identity-residual gradient is written: the shift_out backward
        # forms dS while staging, gcn_dx_finish forms dout*(out > 0)
        fo = {}
        (dA, coefA), gt = tcn_core_backward(unit.tcn1, ts, None, materialize_dx=False,
                                            gpre=(dout, s.out, coef2), gcn_z=_gcn_z(unit, s),
                                            out=fo, off=off)
        g.update({"tcn1." + k: v for k, v in gt.items()})
        extra = {}
        dx, gg = gcn_backward(unit.gcn1, s.gs, dA,
                              extra_dx=(dout, s.out) if kind == "identity" else None,
                              dy_coef=coefA, prev=None if s.prev is None else s.prev[0],
                              extra_out=extra, pre6=fo.get("pre6"), off=off)
        if s.prev is not None:
            s.prev[1].__dict__["_bwd_part"] = (dx, extra["prev_part"])
        g.update({"gcn1." + k: v for k, v in gg.items()})
        return dx, g
    dS = torch.empty_like(S)
    dres = None
    if kind == "conv":
        coefR, g["residual.bn.weight"], g["residual.bn.bias"] = ops.bn_bwd_finalize(
            rpart, B, Cout, B * To * V, s.rs.rst, unit.residual.bn)
        dres = torch.empty_like(s.rs.Rc)
        ops.bn_bwd_apply(dout, s.out, True, S, coef2, False, r=s.rs.Rc, rcoef=coefR, dr=dres,
                         dx=dS)
    elif kind == "identity":
        dres = torch.empty_like(s.x)
        ops.bn_bwd_apply(dout, s.out, True, S, coef2, False, dr=dres, dx=dS)
    else:
        ops.bn_bwd_apply(dout, s.out, True, S, coef2, False, dx=dS)
    fo = {}
    (dA, coefA), gt = tcn_core_backward(unit.tcn1, ts, dS, materialize_dx=False,
                                        gcn_z=_gcn_z(unit, s), out=fo, off=off)
    g.update({"tcn1." + k: v for k, v in gt.items()})
    extra = {}
    dx, gg = gcn_backward(unit.gcn1, s.gs, dA, extra_dx=dres if kind == "identity" else None,
                          dy_coef=coefA, prev=None if s.prev is None else s.prev[0],
                          extra_out=extra, pre6=fo.get("pre6"), off=off)
    if s.prev is not None:   # kind != "conv" and no gcn down conv: dx is final here
        s.prev[1].__dict__["_bwd_part"] = (dx, extra["prev_part"])
    g.update({"gcn1." + k: v for k, v in gg.items()})
    if kind == "conv":
        gr = convbn_dx_and_dw(unit.residual, s.rs, dres, dx, accumulate=True, off=off)
        g.update({"residual." + k: v for k, v in gr.items()})
    return dx, g


# ======================================================================================
# autograd Functions (module forward -> Function.apply(module, input, *params))
# ======================================================================================
# Shift_tcn's shift_in fused into temporal_linear's operand staging (sgcn_pw_fwd_tshift)
# from this many input channels up; below, the two-launch form (shift launch + contraction).
# On gfx950 the fp32 MFMA shares the VALU issue, so the fused operand's per-element tap
# arithmetic comes out of the MFMA budget: with the weight gradients on the side stream
# fusing the C = 128 units cost 0.3 % and C = 256 was neutral (round 2,
# profiles/r02_close/ab_tshift_fusion.txt); since the padded shift kernel (round 3) the
# two-launch form is faster at C = 256 too (+0.5 % same-box, profiles/r03_tsh/), so by
# default no unit fuses (512 exceeds every Shift-GCN width). A/B knob (0 = every unit).
TSHIFT_FUSION_MIN_C = int(os.environ.get("SGCN_TSHIFT_FUSION_MIN_C", "512"))
# The fused operand's two-tap form for channels with |xpos| < 2^-25 (ops.pw_fwd_tshift
# two_row; round 6): 2 = also 0 < xpos < 2^-25 (within 3e-8 x max|tap|), 1 = xpos in
# (-2^-25, 0] only (bit-identical), 0 = four taps always. A/B knob.
TSHIFT_TWO_ROW = int(os.environ.get("SGCN_TSHIFT_TWO_ROW", "2"))
# Inference: the eval-mode BatchNorm right after a conv (down.1 after down.0, residual.bn
# after residual.conv) folded into that conv's weights and bias (folded_conv_bn), so the
# consumer adds the residual without an affine. A/B knob (round 4).
EVAL_FOLD = int(os.environ.get("SGCN_EVAL_FOLD", "1"))
# Shift_gcn.bn's backward sums made by the Shift_tcn.shift_in backward launch
# (sgcn_tshift_bwd_gbn) instead of a separate sgcn_bn_bwd_reduce pass: 2 = every unit (with a
# down conv, the down BatchNorm's sums too; round 3), 1 = units without a down conv only
# (round 2), 0 = off. A/B knob.
GBN_FUSION = int(os.environ.get("SGCN_GBN_FUSION", "2"))
# Off-critical-path launches of linked units on a side stream (_OffPath): the weight-
# gradient contractions (after the dX contraction of the same operand), the position-
# gradient finalizes, the next unit's mask and the forward's down / residual conv branches.
# SGCN_ASYNC_DW=0 serializes everything (bench.py's roofline steps, A/B).
ASYNC_DW = int(os.environ.get("SGCN_ASYNC_DW", "1"))


def trainable(module):
    return [(n, p) for n, p in module.named_parameters() if p.requires_grad]


class _BlockFunction(torch.autograd.Function):
    """Generic Function: ``fwd(module, x, training) -> (y, saved)`` and
    ``bwd(module, saved, dy) -> (dx, {param_name: grad})``.

    The block's input and output are registered with ``save_for_backward`` so autograd's
    version counters guard them: an in-place op on either between forward and backward
    (e.g. ``y.relu_()``) raises autograd's usual "modified by an inplace operation" error
    instead of silently corrupting the ReLU-mask / BatchNorm backward. The fused recipe's
    other saved activations are private (never returned) and are released after the first
    backward; a second backward through the same graph raises a clear error."""

    @staticmethod
    def forward(ctx, impl, module, x, *params):
        fwd, bwd = impl
        training = module.training
        y, saved = fwd(module, x.contiguous(), training)
        ctx.impl, ctx.module, ctx.saved, ctx.training = impl, module, saved, training
        tr = trainable(module)
        ctx.names, ctx.params = [n for n, _ in tr], [p for _, p in tr]
        ctx.save_for_backward(x, y)
        return y

    @staticmethod
    def backward(ctx, dy):
        # eval-mode blocks back-propagate through their running-statistics BatchNorms
        # (fixed affine maps); the BnStats objects saved by the forward carry the mode
        ctx.saved_tensors   # version check of the block's input and output
        if ctx.saved is None:
            raise RuntimeError(
                f"{type(ctx.module).__name__}: backward through the fused HIP block was "
                "called a second time; its saved activations are released after the first "
                "backward (retain_graph=True / double backward is not supported)")
        _, bwd = ctx.impl
        dx, grads = bwd(ctx.module, ctx.saved, dy.contiguous())
        ctx.saved = None
        out = []
        for n, p in zip(ctx.names, ctx.params):
            g = grads.get(n)
            if isinstance(g, _Later):   # written after this returns: accumulated by _finish
                _task(g.t.device).grads.append((p, g.t))
                g = None
            out.append(g)
        return (None, None, dx) + tuple(out)


class _InferFlag(threading.local):
    active = False


# set while a block runs with no backward possible (grad disabled, or nothing requires
# grad; autograd Functions always run forward with grad disabled, so it is decided here):
# eval-mode blocks may then skip tensors only a backward would read
_INFER = _InferFlag()


def run_block(impl, module, x):
    params = [p for _, p in trainable(module)]
    prev = _INFER.active
    _INFER.active = not (torch.is_grad_enabled() and
                         (x.requires_grad or any(p.requires_grad for p in params)))
    try:
        return _BlockFunction.apply(impl, module, x, *params)
    finally:
        _INFER.active = prev


def _gcn_standalone_bwd(mod, s, dy):
    return gcn_backward(mod, s, dy)


def _tcn_standalone_fwd(mod, H, training):
    S, sst, ts = tcn_core_forward(mod, H, training)
    y = ops.bn_apply(S, sst, False)
    return y, ts


def _tcn_standalone_bwd(mod, ts, dy):
    S = ts.S
    B, C, To, V = S.shape
    part, _ = ops.bn_bwd_reduce(dy, None, False, S, ts.sst, False)
    coef, dg, db = ops.bn_bwd_finalize(part, B, C, B * To * V, ts.sst, mod.bn2)
    dS = ops.bn_bwd_apply(dy, None, False, S, coef, False)
    dH, g = tcn_core_backward(mod, ts, dS)
    g["bn2.weight"], g["bn2.bias"] = dg, db
    return dH, g


def _convbn_standalone_fwd(mod, x, training):
    Rc, rst, s = convbn_core_forward(mod, x, training)
    return ops.bn_apply(Rc, rst, False), s


def _convbn_standalone_bwd(mod, s, dy):
    B, C, To, V = s.Rc.shape
    part, _ = ops.bn_bwd_reduce(dy, None, False, s.Rc, s.rst, False)
    coef, dg, db = ops.bn_bwd_finalize(part, B, C, B * To * V, s.rst, mod.bn)
    dRc = ops.bn_bwd_apply(dy, None, False, s.Rc, coef, False)
    dx = torch.zeros_like(s.x)
    g = convbn_dx_and_dw(mod, s, dRc, dx, accumulate=True)
    g["bn.weight"], g["bn.bias"] = dg, db
    return dx, g


GCN_IMPL = (gcn_forward, _gcn_standalone_bwd)
TCN_IMPL = (_tcn_standalone_fwd, _tcn_standalone_bwd)
CONVBN_IMPL = (_convbn_standalone_fwd, _convbn_standalone_bwd)
UNIT_IMPL = (unit_forward, unit_backward)
