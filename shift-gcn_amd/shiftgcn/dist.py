"""Data parallelism: one process per GPU, batch sharded, ONE bucketed gradient all-reduce
per step over RCCL (``torch.distributed`` backend "nccl" on ROCm) / gloo on CPU.

Replaces the reference's single-process ``nn.DataParallel`` (``main.py:294-299``) with
its exact gradient semantics:

* ordinary parameters: ``nn.DataParallel`` sums the per-replica gradients of the
  global-mean loss, which equals the MEAN of per-rank gradients of per-rank mean losses
  (equal shards) -> all-reduce SUM then x 1/world;
* shift positions (``*.xpos`` / ``*.ypos``): each replica's gradient is already
  sign-normalised (+-0.01, ``applyShiftConstraint``) and DataParallel's ReduceAddCoalesced
  SUMS them (``torch/nn/parallel/_functions.py:31-32``) -> all-reduce SUM, no scaling
  (``shift_grad_rule="sum"``, the default; ``"mean"`` is offered as an option);
* BatchNorm uses per-replica batch statistics (no SyncBN), as DataParallel does; the
  running statistics DataParallel keeps are replica 0's -> :func:`broadcast_buffers`
  from rank 0 before evaluation / checkpointing.

The 693,107 fp32 gradients (2.77 MB) go in ONE flat bucket: on MI355X xGMI the ring
all-reduce of 2.77 MB is latency-dominated (tens of us) against >= 9 ms of compute per
step, so one collective after backward is the right shape (no per-layer buckets).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def is_shift_position(name: str) -> bool:
    return name.endswith(".xpos") or name.endswith(".ypos") or name in ("xpos", "ypos")


def trainable_named(model: torch.nn.Module):
    """The parameters that take part in the reduction (the int64 ``shift_in``/``shift_out``
    index arrays are ``requires_grad=False`` and never get a gradient)."""
    return [(n, p) for n, p in model.named_parameters() if p.requires_grad]


def reduction_scale(named, world: int, shift_grad_rule: str = "sum") -> torch.Tensor:
    """Per-element factor applied to the all-reduced SUM of the flat gradient bucket:
    ``1/world`` for ordinary parameters (DataParallel's sum of replica gradients of the
    global-mean loss == mean of per-rank local-mean-loss gradients, equal shards) and 1 for
    shift positions under the default ``"sum"`` rule (DataParallel reduce-adds each
    replica's already sign-normalised +-0.01, ``_functions.py:31-32``)."""
    if shift_grad_rule not in ("sum", "mean"):
        raise ValueError(shift_grad_rule)
    total = sum(p.numel() for _, p in named)
    scale = torch.empty(total, dtype=torch.float32)
    off = 0
    for n, p in named:
        k = p.numel()
        keep_sum = is_shift_position(n) and shift_grad_rule == "sum"
        scale[off:off + k] = 1.0 if keep_sum else 1.0 / world
        off += k
    return scale


def combine_local(grads_per_rank, named, shift_grad_rule: str = "sum"):
    """What :class:`GradAllReduce` leaves in every rank's ``.grad`` given each rank's local
    gradients (a list over ranks of {name: grad}), computed in one process: the SUM over
    ranks (rank order) times :func:`reduction_scale`. Used to check a set of shard passes
    against the DataParallel emulation without a process group."""
    world = len(grads_per_rank)
    scale = reduction_scale(named, world, shift_grad_rule)
    flat = None
    for g in grads_per_rank:
        f = torch.cat([g[n].reshape(-1).float().cpu() for n, _ in named])
        flat = f if flat is None else flat + f
    flat = flat * scale
    out, off = {}, 0
    for n, p in named:
        k = p.numel()
        out[n] = flat[off:off + k].view(p.shape)
        off += k
    return out


class GradAllReduce:
    """Callable run between ``backward()`` and ``optimizer.step()``.

    The flat bucket IS the gradient storage: every trainable parameter's slot is registered
    with the HIP path (``ops.register_grad_slots``), whose backward writes each gradient
    straight into its slot as the tensor autograd then takes as ``.grad`` (no gather into
    the bucket, no copy back). A ``.grad`` that is not its slot (a gradient torch made, one
    set by hand, or an accumulation into fresh memory) is copied in, and every ``.grad``
    is left as its slot. Then ONE all-reduce of the bucket, and the DataParallel scale:
    applied here (one multiply), or, with ``defer_scale_to`` = a :class:`FusedSGD`, inside
    that optimizer's update launch (flags bit 1 of ``sgcn_sgd_step``), which also stores the
    scaled gradient back, so ``.grad`` ends the step holding the same values either way. In
    the deferred form ``.grad`` holds the rank SUM between this call and ``step()``: read or
    clip gradients there only through :meth:`clip_grad_norm_` (or use the immediate form),
    never with a plain ``clip_grad_norm_`` over ``.grad``."""

    def __init__(self, model: torch.nn.Module, group=None, shift_grad_rule: str = "sum",
                 defer_scale_to=None):
        from . import ops
        self.group = group
        self.world = dist.get_world_size(group)
        self.named = trainable_named(model)
        dev = self.named[0][1].device
        self.sizes = [p.numel() for _, p in self.named]
        self.total = sum(self.sizes)
        self.scale = reduction_scale(self.named, self.world, shift_grad_rule).to(dev)
        # per-parameter factor (the rule is per tensor): 1/world, or 1 for summed positions
        self.param_scale = [1.0 if (is_shift_position(n) and shift_grad_rule == "sum")
                            else 1.0 / self.world for n, _ in self.named]
        self.flat = torch.zeros(self.total, dtype=torch.float32, device=dev)
        self.offsets = ops.register_grad_slots(self.named, self.flat)
        self.defer_to = defer_scale_to
        if defer_scale_to is not None and not hasattr(defer_scale_to, "defer_grad_scale"):
            raise TypeError("defer_scale_to must be a shiftgcn.train.FusedSGD")
        self.copied = 0   # gradients copied into the bucket by the last call (diagnostics)
        self.bucket_bytes = 4 * self.total
        self._events = None   # [(start, end)] HIP events around each all_reduce (timing())

    def __call__(self):
        from . import ops
        base = self.flat.data_ptr()
        copied = 0
        for (_, p), off, k in zip(self.named, self.offsets, self.sizes):
            g = p.grad
            if g is not None and g.data_ptr() == base + 4 * off and g.is_contiguous():
                continue   # written in place by the HIP backward
            slot = self.flat[off:off + k].view(p.shape)
            if g is None:
                slot.zero_()
            else:
                slot.copy_(g)
                copied += 1
            p.grad = slot
        self.copied = copied
        # the slots may be handed out again by the next backward (ops.grad_like)
        ops.release_grad_slots([p for _, p in self.named])
        ev = self._events
        if ev is not None:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=self.group)
        if ev is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            ev.append((e0, e1))
        if self.defer_to is not None:
            self.defer_to.defer_grad_scale(
                [(p, s) for (_, p), s in zip(self.named, self.param_scale) if s != 1.0])
        else:
            self.flat.mul_(self.scale)

    def timing(self, on: bool = True):
        """Start (clear) or stop recording HIP events on the current stream around every
        all_reduce: from the moment the stream reaches the collective (its bucket written)
        to the moment the reduced bucket is usable on it, i.e. what the step spends in the
        collective, waiting for slower ranks included."""
        self._events = [] if on else None

    def timing_summary(self):
        """{allreduce_ms_per_step, bucket_bytes, allreduce_bus_gbs, allreduce_calls} over the
        recorded calls (after a device sync); bus GB/s = 2 (world - 1) / world x bytes / time,
        the ring all-reduce convention of nccl-tests / rccl-tests."""
        ev = self._events or []
        if not ev:
            return {"allreduce_ms_per_step": None, "bucket_bytes": self.bucket_bytes,
                    "allreduce_bus_gbs": None, "allreduce_calls": 0}
        ms = sum(a.elapsed_time(b) for a, b in ev) / len(ev)
        bus = 2.0 * (self.world - 1) / self.world * self.bucket_bytes / (ms * 1e-3) / 1e9
        return {"allreduce_ms_per_step": round(ms, 4), "bucket_bytes": self.bucket_bytes,
                "allreduce_bus_gbs": round(bus, 2), "allreduce_calls": len(ev)}

    def clip_grad_norm_(self, max_norm: float, eps: float = 1e-6):
        """``torch.nn.utils.clip_grad_norm_`` (2-norm) of the REDUCED gradients, right after
        this call and before ``step()``, in both scale forms: with ``defer_scale_to`` the
        bucket still holds the rank SUM, so the norm is taken of sum x scale and the clip
        coefficient multiplies the bucket (the deferred scale follows in the update).
        Returns the total norm (a device tensor)."""
        g = self.flat * self.scale if self.defer_to is not None else self.flat
        total = torch.linalg.vector_norm(g)
        self.flat.mul_(torch.clamp(max_norm / (total + eps), max=1.0))
        return total

    def close(self):
        """Unregister the bucket slots (the model's gradients go to fresh memory again)."""
        from . import ops
        ops.unregister_grad_slots([p for _, p in self.named])


def broadcast_buffers(model: torch.nn.Module, src: int = 0, group=None):
    """Make every rank hold rank ``src``'s BatchNorm running statistics (DataParallel keeps
    replica 0's)."""
    from .ops import bump_versions
    bufs = list(model.buffers())
    for b in bufs:
        dist.broadcast(b, src, group=group)
    bump_versions(bufs)   # (eval-mode caches keyed on the running statistics' versions)


def broadcast_parameters(model: torch.nn.Module, src: int = 0, group=None):
    from .ops import bump_versions
    ps = list(model.parameters())
    for p in ps:
        dist.broadcast(p.data, src, group=group)
    bump_versions(ps)
