"""PyTorch-eager CPU restatement of the Shift-GCN model (TEST INFRASTRUCTURE ONLY).

Restates ``model/shift_gcn.py`` (reference) on the CPU with the numpy temporal-shift
restatement of :mod:`oracle.shift_oracle` in place of the ``shift_cuda`` extension:

* :class:`ShiftFunction` / :class:`Shift`  <- ``model/Temporal_shift/cuda/shift.py:9-46``
* :class:`tcn`                             <- ``model/shift_gcn.py:31-45``
* :class:`Shift_tcn`                       <- ``model/shift_gcn.py:48-74``
* :class:`Shift_gcn`                       <- ``model/shift_gcn.py:77-142``
* :class:`TCN_GCN_unit`                    <- ``model/shift_gcn.py:145-162``
* :class:`Model`                           <- ``model/shift_gcn.py:165-216``
* :func:`sgd_param_groups`                 <- ``main.py:301-322`` (per-parameter weight decay)

Parameter names, shapes and dtypes match the reference state_dict, so the same
state_dict loads into the reference model, this oracle and the HIP product model.

Pinned against the imported reference modules by ``tests/golden/gen_fixtures.py``
(committed fixtures; ``tests/test_oracle_model.py``).

It is also the ``cpu_baseline`` ("port") that ``bench.py`` times on the host cores.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn as nn

from . import shift_oracle as so


# --------------------------------------------------------------------------------------
# Temporal shift (shift.py) on the numpy restatement of shift_cuda_kernel.cu
# --------------------------------------------------------------------------------------
class ShiftFunction(torch.autograd.Function):
    """``shift.py:9-30`` with ``shift_cuda.forward/backward`` replaced by the oracle."""

    @staticmethod
    def forward(ctx, inp, xpos, ypos, stride=1):
        inp = inp.contiguous()
        ypos_eff = ypos if stride == 1 else ypos + 0.5          # shift.py:14-18 (fp32 add)
        out = so.shift_forward(inp.detach().numpy(), xpos.detach().numpy(),
                               ypos_eff.detach().numpy(), stride)
        out = torch.from_numpy(out)
        ctx.save_for_backward(inp, xpos, ypos_eff)
        ctx.stride = stride
        return out

    @staticmethod
    def backward(ctx, grad_out):
        inp, xpos, ypos_eff = ctx.saved_tensors
        gin, gx, gy = so.shift_backward(grad_out.contiguous().numpy(), inp.numpy(),
                                        xpos.detach().numpy(), ypos_eff.detach().numpy(),
                                        ctx.stride)
        return torch.from_numpy(gin), torch.from_numpy(gx), torch.from_numpy(gy), None


class Shift(nn.Module):
    """``shift.py:32-46``: owns per-channel ``xpos``/``ypos``. ``function`` is the autograd
    Function standing in for ``ShiftFunction`` (the numpy restatement by default; the
    full-size GPU parity tests swap in a torch-on-device restatement)."""

    function = ShiftFunction

    def __init__(self, channel, stride, init_scale=3):
        super().__init__()
        self.stride = stride
        self.xpos = nn.Parameter(torch.zeros(channel))
        self.ypos = nn.Parameter(torch.zeros(channel))
        self.xpos.data.uniform_(-1e-8, 1e-8)
        self.ypos.data.uniform_(-init_scale, init_scale)

    def forward(self, x):
        return self.function.apply(x, self.xpos, self.ypos, self.stride)


# --------------------------------------------------------------------------------------
# Blocks (shift_gcn.py)
# --------------------------------------------------------------------------------------
def _conv_init(conv):
    nn.init.kaiming_normal_(conv.weight, mode="fan_out")
    nn.init.constant_(conv.bias, 0)


def _bn_init(bn, scale):
    nn.init.constant_(bn.weight, scale)
    nn.init.constant_(bn.bias, 0)


class tcn(nn.Module):  # noqa: N801 (reference name)
    """``shift_gcn.py:31-45``: conv (k x 1, stride (s,1)) + BN2d."""

    def __init__(self, in_channels, out_channels, kernel_size=9, stride=1):
        super().__init__()
        pad = (kernel_size - 1) // 2
        self.conv = nn.Conv2d(in_channels, out_channels, kernel_size=(kernel_size, 1),
                              padding=(pad, 0), stride=(stride, 1))
        self.bn = nn.BatchNorm2d(out_channels)
        self.relu = nn.ReLU()
        _conv_init(self.conv)
        _bn_init(self.bn, 1)

    def forward(self, x):
        return self.bn(self.conv(x))


class Shift_tcn(nn.Module):  # noqa: N801
    """``shift_gcn.py:48-74``: bn -> Shift(s=1) -> 1x1 conv -> ReLU -> Shift(s) -> bn2."""

    def __init__(self, in_channels, out_channels, kernel_size=9, stride=1):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.bn = nn.BatchNorm2d(in_channels)
        self.bn2 = nn.BatchNorm2d(in_channels)
        _bn_init(self.bn2, 1)
        self.relu = nn.ReLU(inplace=True)
        self.shift_in = Shift(channel=in_channels, stride=1, init_scale=1)
        self.shift_out = Shift(channel=out_channels, stride=stride, init_scale=1)
        self.temporal_linear = nn.Conv2d(in_channels, out_channels, 1)
        nn.init.kaiming_normal_(self.temporal_linear.weight, mode="fan_out")

    def forward(self, x):
        x = self.bn(x)
        x = self.shift_in(x)
        x = self.temporal_linear(x)
        x = self.relu(x)
        x = self.shift_out(x)
        return self.bn2(x)


def spatial_shift_indices(num_point: int, channels: int, direction: int) -> np.ndarray:
    """Index arrays of ``shift_gcn.py:108-118`` in closed form.

    ``direction=+1`` (shift_in):  ``idx[i*C+j] = (i*C + j + j*C) mod (C*V) = ((i+j) mod V)*C + j``
    ``direction=-1`` (shift_out): ``idx[i*C+j] = (i*C + j - j*C) mod (C*V) = ((i-j) mod V)*C + j``
    (Python floor-mod: always non-negative). int64, like ``np.empty(...).astype(int)``."""
    i = np.arange(num_point, dtype=np.int64)[:, None]
    j = np.arange(channels, dtype=np.int64)[None, :]
    idx = (i * channels + j + direction * j * channels) % (channels * num_point)
    return idx.reshape(-1).astype(np.int64)


class Shift_gcn(nn.Module):  # noqa: N801
    """``shift_gcn.py:77-142``: joint shift-in gather, feature mask, C_in x C_out linear,
    bias, joint shift-out gather, BN1d(V*C_out), + down(x0), ReLU."""

    def __init__(self, in_channels, out_channels, A, coff_embedding=4, num_subset=3,
                 num_point=25):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        if in_channels != out_channels:
            self.down = nn.Sequential(nn.Conv2d(in_channels, out_channels, 1),
                                      nn.BatchNorm2d(out_channels))
        else:
            self.down = lambda x: x
        self.Linear_weight = nn.Parameter(torch.zeros(in_channels, out_channels))
        nn.init.normal_(self.Linear_weight, 0, math.sqrt(1.0 / out_channels))
        self.Linear_bias = nn.Parameter(torch.zeros(1, 1, out_channels))
        self.Feature_Mask = nn.Parameter(torch.zeros(1, num_point, in_channels))
        self.bn = nn.BatchNorm1d(num_point * out_channels)
        self.relu = nn.ReLU()
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                _conv_init(m)
            elif isinstance(m, nn.BatchNorm2d):
                _bn_init(m, 1)
        self.shift_in = nn.Parameter(
            torch.from_numpy(spatial_shift_indices(num_point, in_channels, +1)),
            requires_grad=False)
        self.shift_out = nn.Parameter(
            torch.from_numpy(spatial_shift_indices(num_point, out_channels, -1)),
            requires_grad=False)

    def forward(self, x0):
        n, c, t, v = x0.size()
        x = x0.permute(0, 2, 3, 1).contiguous().view(n * t, v * c)
        x = torch.index_select(x, 1, self.shift_in).view(n * t, v, c)
        x = x * (torch.tanh(self.Feature_Mask) + 1)
        x = torch.einsum("nwc,cd->nwd", x, self.Linear_weight).contiguous()
        x = x + self.Linear_bias
        x = torch.index_select(x.view(n * t, -1), 1, self.shift_out)
        x = self.bn(x)
        x = x.view(n, t, v, self.out_channels).permute(0, 3, 1, 2)
        x = x + self.down(x0)
        return self.relu(x)


class TCN_GCN_unit(nn.Module):  # noqa: N801
    """``shift_gcn.py:145-162``: relu(tcn1(gcn1(x)) + residual(x))."""

    def __init__(self, in_channels, out_channels, A, stride=1, residual=True,
                 num_point=25):
        super().__init__()
        self.gcn1 = Shift_gcn(in_channels, out_channels, A, num_point=num_point)
        self.tcn1 = Shift_tcn(out_channels, out_channels, stride=stride)
        self.relu = nn.ReLU()
        if not residual:
            self.residual = lambda x: 0
        elif in_channels == out_channels and stride == 1:
            self.residual = lambda x: x
        else:
            self.residual = tcn(in_channels, out_channels, kernel_size=1, stride=stride)

    def forward(self, x):
        return self.relu(self.tcn1(self.gcn1(x)) + self.residual(x))


UNIT_PLAN = (  # (C_in, C_out, stride, residual) for l1..l10 (shift_gcn.py:178-187)
    (3, 64, 1, False), (64, 64, 1, True), (64, 64, 1, True), (64, 64, 1, True),
    (64, 128, 2, True), (128, 128, 1, True), (128, 128, 1, True),
    (128, 256, 2, True), (256, 256, 1, True), (256, 256, 1, True),
)


class Model(nn.Module):
    """``shift_gcn.py:165-216`` (graph object is unused by the compute path)."""

    def __init__(self, num_class=60, num_point=25, num_person=2, graph=None,
                 graph_args=dict(), in_channels=3):  # noqa: B006 (reference signature)
        super().__init__()
        self.data_bn = nn.BatchNorm1d(num_person * in_channels * num_point)
        for k, (ci, co, s, r) in enumerate(UNIT_PLAN, start=1):
            if k == 1:
                ci = in_channels
            setattr(self, f"l{k}", TCN_GCN_unit(ci, co, None, stride=s, residual=r,
                                                num_point=num_point))
        self.fc = nn.Linear(256, num_class)
        nn.init.normal_(self.fc.weight, 0, math.sqrt(2.0 / num_class))
        _bn_init(self.data_bn, 1)

    def forward(self, x):
        N, C, T, V, M = x.size()
        x = x.permute(0, 4, 3, 1, 2).contiguous().view(N, M * V * C, T)
        x = self.data_bn(x)
        x = x.view(N, M, V, C, T).permute(0, 1, 3, 4, 2).contiguous().view(N * M, C, T, V)
        for k in range(1, 11):
            x = getattr(self, f"l{k}")(x)
        c_new = x.size(1)
        x = x.view(N, M, c_new, -1).mean(3).mean(1)
        return self.fc(x)


def sgd_param_groups(model: nn.Module, base_lr: float):
    """``main.py:301-322``: one group per named parameter; weight decay 1e-3 for
    ``*Linear_weight*``, 0 for ``*Mask*``, else 1e-4 (biases and shift positions too)."""
    groups = []
    for key, value in model.named_parameters():
        wd = 1e-4
        if "Linear_weight" in key:
            wd = 1e-3
        elif "Mask" in key:
            wd = 0.0
        groups.append({"params": value, "lr": base_lr, "weight_decay": wd})
    return groups
