"""Drop-in for ``model/shift_gcn.py`` on the MI355X HIP path.

Same class names, constructor signatures, submodule/parameter names, shapes and dtypes
as the reference (``shift_gcn.py:14-216``), so reference checkpoints load unchanged
(``main.py:219``, ``inference_pipeline.py:331-337``). The forward passes of
``Shift_gcn``, ``Shift_tcn``, ``tcn`` (kernel_size=1) and ``TCN_GCN_unit`` run the fused
HIP recipes of :mod:`shiftgcn.fused`; there is no CPU path (CPU tensors raise like the
reference's ``CHECK_INPUT``).

``Model``'s input permute + ``data_bn`` and the global average pool run the HIP kernels of
:mod:`shiftgcn.head`; the classifier ``fc`` is ``nn.Linear`` (a library
GEMM on the device). ``tcn`` with kernel_size != 1 (never instantiated by ``Model``) uses
``torch.nn.functional.conv2d`` on the device.
"""
from __future__ import annotations

import contextlib
import importlib
import math

import numpy as np
import torch
import torch.nn as nn

from . import fused, head
from .shift import Shift


def import_class(name):
    """``shift_gcn.py:14-19`` (dotted path -> attribute)."""
    components = name.split(".")
    mod = importlib.import_module(components[0])
    for comp in components[1:]:
        try:
            mod = getattr(mod, comp)
        except AttributeError:
            mod = importlib.import_module(mod.__name__ + "." + comp)
    return mod


def conv_init(conv):
    nn.init.kaiming_normal_(conv.weight, mode="fan_out")
    nn.init.constant_(conv.bias, 0)


def bn_init(bn, scale):
    nn.init.constant_(bn.weight, scale)
    nn.init.constant_(bn.bias, 0)


def _default_device():
    return "cuda" if torch.cuda.is_available() else "cpu"


class tcn(nn.Module):  # noqa: N801 (reference name)
    """``shift_gcn.py:31-45``: Conv2d (k x 1, stride (s,1)) + BatchNorm2d."""

    def __init__(self, in_channels, out_channels, kernel_size=9, stride=1):
        super().__init__()
        pad = int((kernel_size - 1) / 2)
        self.conv = nn.Conv2d(in_channels, out_channels, kernel_size=(kernel_size, 1),
                              padding=(pad, 0), stride=(stride, 1))
        self.bn = nn.BatchNorm2d(out_channels)
        self.relu = nn.ReLU()
        conv_init(self.conv)
        bn_init(self.bn, 1)
        self.kernel_size = kernel_size
        self.stride = stride

    def forward(self, x):
        if self.kernel_size == 1:
            return fused.run_block(fused.CONVBN_IMPL, self, x)
        return self.bn(self.conv(x))  # not on the hot path (never built by Model)


class Shift_tcn(nn.Module):  # noqa: N801
    """``shift_gcn.py:48-74``: bn -> Shift(s=1) -> 1x1 conv -> ReLU -> Shift(s) -> bn2."""

    def __init__(self, in_channels, out_channels, kernel_size=9, stride=1):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.bn = nn.BatchNorm2d(in_channels)
        self.bn2 = nn.BatchNorm2d(in_channels)
        bn_init(self.bn2, 1)
        self.relu = nn.ReLU(inplace=True)
        self.shift_in = Shift(channel=in_channels, stride=1, init_scale=1)
        self.shift_out = Shift(channel=out_channels, stride=stride, init_scale=1)
        self.temporal_linear = nn.Conv2d(in_channels, out_channels, 1)
        nn.init.kaiming_normal_(self.temporal_linear.weight, mode="fan_out")

    def forward(self, x):
        return fused.run_block(fused.TCN_IMPL, self, x)


class Shift_gcn(nn.Module):  # noqa: N801
    """``shift_gcn.py:77-142``. ``A``, ``coff_embedding`` and ``num_subset`` are accepted
    and unused, as in the reference."""

    def __init__(self, in_channels, out_channels, A, coff_embedding=4, num_subset=3,
                 num_point=25):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.num_point = num_point
        self.has_down = in_channels != out_channels
        if self.has_down:
            self.down = nn.Sequential(nn.Conv2d(in_channels, out_channels, 1),
                                      nn.BatchNorm2d(out_channels))
        else:
            self.down = lambda x: x
        dev = _default_device()
        self.Linear_weight = nn.Parameter(torch.zeros(in_channels, out_channels, device=dev))
        nn.init.normal_(self.Linear_weight, 0, math.sqrt(1.0 / out_channels))
        self.Linear_bias = nn.Parameter(torch.zeros(1, 1, out_channels, device=dev))
        self.Feature_Mask = nn.Parameter(torch.zeros(1, num_point, in_channels, device=dev))
        self.bn = nn.BatchNorm1d(num_point * out_channels)
        self.relu = nn.ReLU()
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                conv_init(m)
            elif isinstance(m, nn.BatchNorm2d):
                bn_init(m, 1)
        # shift_gcn.py:108-118 in closed form (Python floor-mod), int64, requires_grad=False
        i = np.arange(num_point, dtype=np.int64)[:, None]
        self.shift_in = nn.Parameter(torch.from_numpy(
            ((i * in_channels + np.arange(in_channels) * (1 + in_channels))
             % (in_channels * num_point)).reshape(-1)), requires_grad=False)
        self.shift_out = nn.Parameter(torch.from_numpy(
            ((i * out_channels + np.arange(out_channels) * (1 - out_channels))
             % (out_channels * num_point)).reshape(-1)), requires_grad=False)

    def forward(self, x0):
        return fused.run_block(fused.GCN_IMPL, self, x0)


class TCN_GCN_unit(nn.Module):  # noqa: N801
    """``shift_gcn.py:145-162``: relu(tcn1(gcn1(x)) + residual(x)) as one fused block."""

    def __init__(self, in_channels, out_channels, A, stride=1, residual=True, num_point=25):
        super().__init__()
        self.gcn1 = Shift_gcn(in_channels, out_channels, A, num_point=num_point)
        self.tcn1 = Shift_tcn(out_channels, out_channels, stride=stride)
        self.relu = nn.ReLU()
        if not residual:
            self.residual = lambda x: 0
            self.residual_kind = "none"
        elif in_channels == out_channels and stride == 1:
            self.residual = lambda x: x
            self.residual_kind = "identity"
        else:
            self.residual = tcn(in_channels, out_channels, kernel_size=1, stride=stride)
            self.residual_kind = "conv"

    def forward(self, x):
        return fused.run_block(fused.UNIT_IMPL, self, x)


class Model(nn.Module):
    """``shift_gcn.py:165-216``."""

    def __init__(self, num_class=60, num_point=25, num_person=2, graph=None,
                 graph_args=dict(), in_channels=3):  # noqa: B006 (reference signature)
        super().__init__()
        if graph is None:
            raise ValueError()
        if isinstance(graph, str):
            try:
                Graph = import_class(graph)
            except ImportError:
                if not graph.startswith("graph."):
                    raise
                Graph = import_class("shiftgcn." + graph)   # bundled graph/ definitions
        else:
            Graph = graph
        self.graph = Graph(**graph_args)
        A = self.graph.A
        self.num_person, self.in_channels = num_person, in_channels
        self.data_bn = nn.BatchNorm1d(num_person * in_channels * num_point)
        self.l1 = TCN_GCN_unit(3, 64, A, residual=False, num_point=num_point)
        self.l2 = TCN_GCN_unit(64, 64, A, num_point=num_point)
        self.l3 = TCN_GCN_unit(64, 64, A, num_point=num_point)
        self.l4 = TCN_GCN_unit(64, 64, A, num_point=num_point)
        self.l5 = TCN_GCN_unit(64, 128, A, stride=2, num_point=num_point)
        self.l6 = TCN_GCN_unit(128, 128, A, num_point=num_point)
        self.l7 = TCN_GCN_unit(128, 128, A, num_point=num_point)
        self.l8 = TCN_GCN_unit(128, 256, A, stride=2, num_point=num_point)
        self.l9 = TCN_GCN_unit(256, 256, A, num_point=num_point)
        self.l10 = TCN_GCN_unit(256, 256, A, num_point=num_point)
        self.fc = nn.Linear(256, num_class)
        nn.init.normal_(self.fc.weight, 0, math.sqrt(2.0 / num_class))
        bn_init(self.data_bn, 1)

    def forward(self, x):
        N, C, T, V, M = x.size()
        # permute -> data_bn -> permute back (:194-198) as one statistics pass + one
        # fused apply pass over the clip
        x = head.data_bn_planes(self.data_bn, x.contiguous())
        return self.forward_planes(x, N, M)

    def forward_planes(self, x, N, M):
        """Body + head of ``forward`` (shift_gcn.py:200-216) on an input already permuted
        to (N*M, C, T, V) and normalised by ``data_bn`` (e.g. by ``sgcn_modalities``)."""
        units = [getattr(self, f"l{k}") for k in range(1, 11)]
        with linked_units(units):
            for u in units:
                x = u(x)
        x = head.pool(x, N, M)        # x.view(N, M, C, -1).mean(3).mean(1)  (:211-214)
        return head.linear(self.fc, x)


@contextlib.contextmanager
def linked_units(units):
    """Run a chain of TCN_GCN_units with the cross-unit fusions on (what Model.forward
    does for l1..l10): each unit's tail launch also writes the next unit's gathered gcn
    input, and the next unit's backward makes this unit's bn2 backward partials. The links
    live only for the duration of the block (a unit used alone runs unfused). Linked units
    also run their weight-gradient contractions on a side stream, joined before
    ``backward()`` returns (fused._OffPath)."""
    try:
        for u, nxt in zip(units[:-1], units[1:]):
            u.__dict__["_gather_consumer"] = nxt.gcn1
            u.__dict__["_next_unit"] = nxt
        for i, u in enumerate(units):
            if i or not fused.TAIL_MAIN & 2:
                u.__dict__["_off_path"] = True
        # every unit's tanh(Feature_Mask) + 1 in one launch (fused.prepare_masks)
        fused.prepare_masks([u.gcn1 for u in units])
        yield
    finally:
        for u in units:
            u.__dict__.pop("_gather_consumer", None)
            u.__dict__.pop("_next_unit", None)
            u.__dict__.pop("_off_path", None)
            u.__dict__.pop("_prev_tail", None)
            u.gcn1.__dict__.pop("_gather_cache", None)
            u.gcn1.__dict__.pop("_mask_ready", None)
