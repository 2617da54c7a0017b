"""Single-process restatement of the reference's ``nn.DataParallel`` training semantics
(TEST INFRASTRUCTURE ONLY: imported by ``tests/`` as the checker, never by the product).

``main.py:294-299`` wraps the model in ``nn.DataParallel(model, device_ids=...)``; one
training iteration (``main.py:397-416``) then does, per step:

* scatter the batch along dim 0 into k equal chunks (``torch/nn/parallel/scatter_gather``);
* replicate the module: replica 0 IS the original module's parameters and buffers (the
  broadcast's source-device outputs are the inputs themselves), replicas 1..k-1 are copies;
* run every replica on its chunk (BatchNorm uses that replica's chunk statistics, no
  SyncBN), gather the logits, take ONE CrossEntropy mean over the whole batch;
* backward: every replica receives the gradient of that global-mean loss; the Broadcast
  backward (``ReduceAddCoalesced``, ``torch/nn/parallel/_functions.py:10-32``) SUMS the
  replicas' parameter gradients onto the original. The temporal-shift positions' gradients
  are sign-normalised per replica by the extension's ``applyShiftConstraint``
  (``shift_cuda_kernel.cu:370-395``) before that sum, so they add up as k x +-0.01;
* running statistics: replica 0's updates land in the original module (the others' are
  discarded).

:func:`dataparallel_grads` computes exactly that with k deep copies on one device.
"""
from __future__ import annotations

import copy

import torch


def dataparallel_grads(model: torch.nn.Module, x: torch.Tensor, labels: torch.Tensor, k: int):
    """Run one DataParallel forward/backward of ``model`` (replica 0 = ``model`` itself,
    so its BN running stats are updated in place like DataParallel's) on ``x`` split into
    ``k`` equal chunks. Returns ``(loss, logits, {name: summed grad})``."""
    assert x.shape[0] % k == 0, "equal shards"
    replicas = [model] + [copy.deepcopy(model) for _ in range(k - 1)]
    for r in replicas:
        r.zero_grad(set_to_none=True)
    chunks = torch.chunk(x, k, dim=0)
    logits = torch.cat([r(c) for r, c in zip(replicas, chunks)], dim=0)
    loss = torch.nn.functional.cross_entropy(logits, labels)
    loss.backward()
    grads = {}
    for name, p in model.named_parameters():
        if not p.requires_grad:
            continue
        acc = None
        for r in replicas:
            g = dict(r.named_parameters())[name].grad
            if g is None:
                continue
            acc = g.clone() if acc is None else acc + g
        grads[name] = acc
    return loss.detach(), logits.detach(), grads
