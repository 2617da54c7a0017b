"""Model head and tail on the HIP path (``shift_gcn.py:193-216``).

* :func:`data_bn_planes` — ``x.permute(0, 4, 3, 1, 2).view(N, M*V*C, T)`` ->
  ``data_bn`` (BatchNorm1d(M*V*C), training or eval semantics of the module, running
  statistics updated like ``nn.BatchNorm1d.forward``) -> planes ``(N*M, C, T, V)``, as
  ``sgcn_head_moments`` + ``sgcn_bn_finalize`` + ``sgcn_head_apply`` (one read of the clip
  for the statistics, one fused permute+apply pass). Backward: ``sgcn_head_bwd_reduce`` +
  ``sgcn_bn_bwd_finalize`` (data_bn's weight/bias gradients) and, only when the clip
  requires a gradient, ``sgcn_head_bwd_apply``.
* :func:`pool` — ``x.view(N, M, C, -1).mean(3).mean(1)`` as ``sgcn_pool`` /
  ``sgcn_pool_bwd``.

The classifier ``fc`` (a (N, 256) x (256, num_class) GEMM) stays ``nn.Linear`` (a library
GEMM on the device).
"""
from __future__ import annotations

import torch

from . import ops


def _batch_stats(bn) -> bool:
    # nn.modules.batchnorm._BatchNorm.forward: bn_training
    return bn.training or (bn.running_mean is None and bn.running_var is None)


class _DataBnFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, bn):
        N, C, T, V, M = x.shape
        F = M * V * C
        if _batch_stats(bn):
            if N * T <= 1:
                # F.batch_norm's check (torch/nn/functional.py _verify_batch_size)
                raise ValueError("Expected more than 1 value per channel when training, got "
                                 f"input size {torch.Size([N, F, T])}")
            st = ops.bn_finalize(ops.head_moments(x), N, F, T, bn, training=bn.training)
        else:
            st = ops.bn_eval_coef(bn, F)
        ctx.save_for_backward(x)
        ctx.st, ctx.bn = st, bn
        return ops.head_apply(x, st)

    @staticmethod
    def backward(ctx, gy):
        (x,) = ctx.saved_tensors
        st, bn = ctx.st, ctx.bn
        N, C, T, V, M = x.shape
        gy = gy.contiguous()
        part = ops.head_bwd_reduce(gy, x, st)
        coef, dgamma, dbeta = ops.bn_bwd_finalize(part, N, M * V * C, N * T, st, bn)
        dx = ops.head_bwd_apply(gy, x, coef) if ctx.needs_input_grad[0] else None
        return (dx, dgamma if ctx.needs_input_grad[1] else None,
                dbeta if ctx.needs_input_grad[2] else None, None)


class _PoolFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, N, M):
        ctx.shape, ctx.N, ctx.M = x.shape, N, M
        return ops.pool(x, N, M)

    @staticmethod
    def backward(ctx, g):
        return ops.pool_bwd(g.contiguous(), ctx.shape, ctx.N, ctx.M), None, None


class _LinearSlotsFunction(torch.autograd.Function):
    """``fc`` (F.linear = addmm(bias, x, weight.t())) whose weight / bias gradients are
    written into their gradient slots (shiftgcn.dist.GradAllReduce's bucket): the same
    calls torch's addmm backward makes (mm_mat2_backward for a column-major mat2:
    ``grad.t().mm(x)``; mm_mat1_backward: ``grad.mm(weight)``; the bias: the sum over the
    batch), with ``out=`` the slot."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.params = (weight, bias)   # the parameters themselves: their slots and .grad
        return torch.nn.functional.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        weight, bias = ctx.params
        dx = g.mm(w) if ctx.needs_input_grad[0] else None
        dw = db = None
        if ctx.needs_input_grad[1]:
            dw = ops.grad_like(weight)
            torch.mm(g.t(), x, out=dw)
        if bias is not None and ctx.needs_input_grad[2]:
            db = ops.grad_like(bias)
            torch.sum(g, 0, out=db)
        return dx, dw, db


def linear(fc, x):
    """``fc(x)``; through :class:`_LinearSlotsFunction` while fc's weight has a gradient
    slot (a data-parallel bucket is registered), so its gradients land in the bucket."""
    if ops.grad_slot(fc.weight) is None or x.dim() != 2:
        return fc(x)
    return _LinearSlotsFunction.apply(x, fc.weight, fc.bias)


def data_bn_planes(bn, x):
    """(N, C, T, V, M) clip -> data_bn-normalised planes (N*M, C, T, V)."""
    ops.check_input(x, "input")
    if x.dim() != 5:
        raise RuntimeError(f"expected a (N, C, T, V, M) clip, got shape {tuple(x.shape)}")
    N, C, T, V, M = x.shape
    if bn.num_features != M * V * C:
        raise RuntimeError(f"data_bn has {bn.num_features} features, the clip {M * V * C}")
    return _DataBnFunction.apply(x, bn.weight, bn.bias, bn)


def pool(x, N, M):
    """Last unit's output (N*M, C, T, V) -> (N, C) global average over (T, V) and M."""
    ops.check_input(x, "input")
    if x.shape[0] != N * M:
        raise RuntimeError(f"expected {N * M} planes, got {x.shape[0]}")
    return _PoolFunction.apply(x, N, M)
