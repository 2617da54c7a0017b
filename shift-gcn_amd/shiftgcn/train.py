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


def build_optimizer(model, base_lr=0.1, nesterov=True, momentum=0.9, merge_groups=True):
    groups = (merged_param_groups if merge_groups else sgd_param_groups)(model, base_lr)
    return torch.optim.SGD(groups, lr=base_lr, momentum=momentum, nesterov=nesterov,
                           foreach=True)


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
