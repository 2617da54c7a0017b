"""Training-step semantics of the reference harness (``main.py``) on the HIP model.

* :func:`sgd_param_groups` — ``main.py:301-322``: one group per named parameter; weight
  decay 1e-3 for ``*Linear_weight*``, 0 for ``*Mask*``, 1e-4 otherwise (biases and the
  shift positions included); SGD momentum 0.9, nesterov per the YAML configs.
* :func:`adjust_learning_rate` — ``main.py:342-353`` (warm-up, step decay x0.1).
* :func:`train_step` — ``main.py:397-416``: forward, CrossEntropy, zero_grad, backward,
  (data-parallel gradient reduction), optimizer step.
"""
from __future__ import annotations

import numpy as np
import torch


def sgd_param_groups(model: torch.nn.Module, base_lr: float):
    groups = []
    for key, value in model.named_parameters():
        if not value.requires_grad:
            continue  # the int64 shift_in/shift_out index arrays never get a gradient
        wd = 1e-4
        if "Linear_weight" in key:
            wd = 1e-3
        elif "Mask" in key:
            wd = 0.0
        groups.append({"params": value, "lr": base_lr, "weight_decay": wd})
    return groups


def merged_param_groups(model: torch.nn.Module, base_lr: float):
    """The same per-parameter hyper-parameters as :func:`sgd_param_groups`, merged into one
    group per weight-decay value (3 groups). SGD's update is per parameter, so this is
    numerically identical, but the multi-tensor (foreach) kernels then cover ~50
    parameters per launch instead of one: ~660 optimizer launches per step -> ~10."""
    by_wd = {}
    for g in sgd_param_groups(model, base_lr):
        by_wd.setdefault(g["weight_decay"], []).append(g["params"])
    return [{"params": ps, "lr": base_lr, "weight_decay": wd} for wd, ps in by_wd.items()]


class _HyperGroup(dict):
    """A FusedSGD parameter group: assigning its ``lr`` / ``weight_decay`` (what
    :func:`adjust_learning_rate` and torch's LR schedulers do) also updates the optimizer's
    device-resident copy, the one a graph-captured step reads at replay."""

    __slots__ = ("_opt",)

    def __init__(self, group, opt):
        super().__init__(group)
        self._opt = opt

    def __setitem__(self, k, v):
        super().__setitem__(k, v)
        if k in ("lr", "weight_decay"):
            self._opt._hyper_changed(self)


class FusedSGD(torch.optim.SGD):
    """``torch.optim.SGD`` (same constructor, param groups, hyper-parameters and state:
    ``state[p]["momentum_buffer"]``, so ``state_dict`` / ``load_state_dict`` round-trip with
    the stock optimizer) whose ``step`` updates every parameter of every group in ONE
    launch (``sgcn_sgd_step``) instead of torch's ~35 multi-tensor launches per step.
    Same arithmetic in the same order as torch's single/multi-tensor SGD (weight decay,
    momentum with the first-step clone, nesterov, update); groups must share momentum,
    dampening 0, nesterov and not maximize — otherwise, and for CPU or non-fp32
    parameters, the stock ``step`` runs. Closures are supported as in torch.

    Under hipGraph capture the launch reads each group's (weight_decay, lr) from a device
    pair the optimizer keeps current (``sgcn_sgd_step`` flags bit 2): assigning
    ``group["lr"]`` between replays (``adjust_learning_rate``, an LR scheduler) writes it
    on the current stream, so the next replay uses the new value (main.py:342-353).
    ``momentum`` / ``nesterov`` are launch arguments and stay those of the capture."""

    def __init__(self, params, lr=1e-3, momentum=0.0, dampening=0.0, weight_decay=0.0,
                 nesterov=False, **kw):
        kw.pop("foreach", None)
        super().__init__(params, lr=lr, momentum=momentum, dampening=dampening,
                         weight_decay=weight_decay, nesterov=nesterov, foreach=True, **kw)
        self._layout = None   # (param signature, device numel / chunk map, n chunks)
        self._gscale = {}     # id(param) -> (param, gradient scale) for the next step only
        self._cap = None      # (pinned table buffer, device table) for a step under capture
        self._hyper = None    # device (groups, 2) float32 {weight_decay, lr}, and its host mirror
        self._hyper_host = None

    def add_param_group(self, param_group):
        super().add_param_group(param_group)
        self._wrap_groups()

    def __setstate__(self, state):   # (also what load_state_dict installs new groups with)
        super().__setstate__(state)
        self._wrap_groups()

    def _wrap_groups(self):
        pg = self.param_groups
        for i, g in enumerate(pg):
            if not isinstance(g, _HyperGroup):
                pg[i] = _HyperGroup(g, self)
        h = getattr(self, "_hyper", None)
        if h is not None:
            if h.shape[0] != len(pg):
                self._hyper = self._hyper_host = None   # re-made by the next eager step
            else:
                for g in pg:
                    self._hyper_changed(g)

    def _hyper_changed(self, group):
        """Write ``group``'s (weight_decay, lr) into the device pair (current stream)."""
        h = getattr(self, "_hyper", None)
        if h is None:
            return
        for i, g in enumerate(self.param_groups):
            if g is group:
                v = (float(g["weight_decay"]), float(g["lr"]))
                if self._hyper_host[i] != v:
                    h[i, 0].fill_(v[0])
                    h[i, 1].fill_(v[1])
                    self._hyper_host[i] = v
                return

    def defer_grad_scale(self, pairs):
        """[(param, s)]: the next ``step`` first scales these parameters' gradients by s
        and stores them back (shiftgcn.dist.GradAllReduce's DataParallel 1/world), inside
        the update launch."""
        self._gscale = {id(p): (p, float(s)) for p, s in pairs}

    def _native_ok(self, items):
        g0 = self.param_groups[0]
        for g in self.param_groups:
            if (g["momentum"] != g0["momentum"] or g["nesterov"] != g0["nesterov"] or
                    g["dampening"] != 0 or g.get("maximize", False) or
                    g.get("differentiable", False)):
                return False
        if len({p.device for p, _ in items}) != 1:
            return False
        for p, _ in items:
            if not (p.is_cuda and p.dtype == torch.float32 and p.grad.dtype == torch.float32
                    and not p.grad.is_sparse and p.is_contiguous() and p.grad.is_contiguous()
                    and p.grad.device == p.device):
                return False
            # an existing momentum buffer goes into the kernel's table as a raw pointer: it
            # must be a float32 contiguous tensor of p's size ON p's device (e.g. state
            # loaded before model.cuda() stays on the host; torch's SGD raises there)
            buf = self.state.get(p, {}).get("momentum_buffer")
            if buf is not None and not (buf.device == p.device and buf.dtype == torch.float32
                                        and buf.is_contiguous() and buf.numel() == p.numel()):
                return False
        return True

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        gscale, self._gscale = self._gscale, {}
        items = [(p, g) for g in self.param_groups for p in g["params"] if p.grad is not None]
        if not items:
            return loss
        if not self._native_ok(items):
            for p, sc in gscale.values():   # the deferred scale as its own multiply
                if p.grad is not None:
                    p.grad.mul_(sc)
            super().step()     # (the closure, if any, was evaluated above)
            return loss
        import struct

        from . import _lib
        from .ops import _stream, bump_versions
        lib = _lib.load()
        g0 = self.param_groups[0]
        momentum = float(g0["momentum"])
        dev = items[0][0].device
        sig = tuple((id(p), p.numel()) for p, _ in items)
        if self._layout is None or self._layout[0] != sig:
            ch = lib.sgcn_sgd_chunk_elems()
            numel = [p.numel() for p, _ in items]
            chunks = [v for t, n in enumerate(numel) for s0 in range(0, n, ch) for v in (t, s0)]
            self._layout = (sig, torch.tensor(numel, dtype=torch.int32, device=dev),
                            torch.tensor(chunks, dtype=torch.int32, device=dev),
                            len(chunks) // 2)
        _, numel_d, chunks_d, nchunks = self._layout
        capturing = torch.cuda.is_current_stream_capturing()
        if capturing:
            # the launch reads (weight_decay, lr) from the device pairs at every replay
            if (self._hyper is None or self._hyper.device != dev or
                    any(hh != (float(g["weight_decay"]), float(g["lr"]))
                        for hh, g in zip(self._hyper_host, self.param_groups))):
                raise RuntimeError("FusedSGD: run one eager step before capturing a graph "
                                   "(and set lr / weight_decay by item assignment)")
        rows = []
        for gi, g in enumerate(self.param_groups):
            if capturing:
                wdlr = self._hyper[gi].data_ptr()
            else:
                wdlr = struct.unpack("<q", struct.pack("<ff", float(g["weight_decay"]),
                                                      float(g["lr"])))[0]
            for p in g["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                first = 0
                if momentum != 0 and st.get("momentum_buffer") is None:
                    st["momentum_buffer"] = torch.empty_like(p, memory_format=torch.preserve_format)
                    first = 1
                buf = st.get("momentum_buffer") if momentum != 0 else p
                flags = first | (4 if capturing else 0)
                sc = gscale.get(id(p))
                if sc is not None and sc[0] is p:
                    # bit 1 + the float's bits in 32-63 (a signed int64 for the table)
                    bits = struct.unpack("<I", struct.pack("<f", sc[1]))[0]
                    flags |= 2 | (bits << 32)
                    flags = struct.unpack("<q", struct.pack("<Q", flags))[0]
                rows += [p.data_ptr(), p.grad.data_ptr(), buf.data_ptr(), wdlr, flags]
        if capturing:
            # hipGraph capture (bench.py --graph): no host allocation is allowed here, so the
            # table goes through a pinned buffer and device table set up by an eager step;
            # the captured copy re-reads the buffer at every replay (same addresses: the
            # graph's gradients and buffers are static; the hyper-parameters are read through
            # the device pairs, flags bit 2)
            if self._cap is None or self._cap[0].numel() != len(rows):
                raise RuntimeError("FusedSGD: run one eager step before capturing a graph")
            host, table = self._cap
            host.numpy()[:] = rows
            table.copy_(host, non_blocking=True)
            from . import ops
            ops.mark_captured_writes()   # the eval caches cannot see replayed updates
        else:
            table = torch.tensor(rows, dtype=torch.int64).pin_memory().to(dev, non_blocking=True)
            if self._cap is None or self._cap[0].numel() != len(rows):
                self._cap = (torch.empty(len(rows), dtype=torch.int64).pin_memory(),
                             torch.empty(len(rows), dtype=torch.int64, device=dev))
            if self._hyper is None or self._hyper.device != dev:
                self._hyper = torch.empty((len(self.param_groups), 2), dtype=torch.float32,
                                          device=dev)
                self._hyper_host = [None] * len(self.param_groups)
            for g in self.param_groups:   # (a no-op unless a value changed without a hook)
                self._hyper_changed(g)
        rc = lib.sgcn_sgd_step(table.data_ptr(), numel_d.data_ptr(), chunks_d.data_ptr(),
                               nchunks, momentum, int(bool(g0["nesterov"])), _stream(table))
        _lib.check(rc, "sgcn_sgd_step")
        # the kernel wrote every parameter, momentum buffer and scaled gradient in place:
        # advance their version counters as torch's own in-place update would
        written = [p for p, _ in items]
        if momentum != 0:
            written += [self.state[p]["momentum_buffer"] for p in written]
        written += [p.grad for p, _ in items if id(p) in gscale]
        bump_versions(written)
        return loss


def build_optimizer(model, base_lr=0.1, nesterov=True, momentum=0.9, merge_groups=True,
                    fused=None):
    """The reference's SGD; ``fused``: the one-launch native update (:class:`FusedSGD`;
    default on, ``SGCN_FUSED_SGD=0`` selects torch's foreach SGD for A/B runs)."""
    if fused is None:
        import os
        fused = os.environ.get("SGCN_FUSED_SGD", "1") != "0"
    groups = (merged_param_groups if merge_groups else sgd_param_groups)(model, base_lr)
    cls = FusedSGD if fused else torch.optim.SGD
    return cls(groups, lr=base_lr, momentum=momentum, nesterov=nesterov, foreach=True)


def adjust_learning_rate(optimizer, epoch, base_lr=0.1, steps=(60, 80, 100), warm_up_epoch=0):
    if epoch < warm_up_epoch:
        lr = base_lr * (epoch + 1) / warm_up_epoch
    else:
        lr = base_lr * (0.1 ** np.sum(epoch >= np.array(steps)))
    for g in optimizer.param_groups:
        g["lr"] = lr
    return lr


def train_step(model, optimizer, x, label, grad_sync=None):
    """One reference training iteration; returns the (device) loss tensor."""
    output = model(x)
    loss = torch.nn.functional.cross_entropy(output, label)
    optimizer.zero_grad(set_to_none=True)
    loss.backward()
    if grad_sync is not None:
        grad_sync()
    optimizer.step()
    return loss
