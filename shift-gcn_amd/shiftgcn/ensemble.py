"""Four-stream ensemble inference (BASELINE config 4) on the HIP path.

Reference: ``inference_pipeline.py:284-309`` (``derive_modalities``: bone / joint-motion /
bone-motion streams from a joint window), ``:342-370`` (``run_ensemble_inference``: one
Model per stream in eval mode, ``ensemble_logits += alpha * logits`` in float64 with
``ENSEMBLE_WEIGHTS_DEFAULT = [0.6, 0.6, 0.4, 0.4]`` (``:24``), softmax, class 1 = fall),
and ``ensemble.py:18-32`` (the same weighted score fusion for the NTU streams).

The reference runs every window through every model at batch 1 and derives the streams
in numpy on the host. Here a whole batch of windows is one ``sgcn_modalities`` launch
(streams derived, permuted into the (N*M, C, T, V) plane layout and ``data_bn`` applied
for all four models in one pass), four batched eval-mode forwards on the fused blocks,
and the fp64 score fusion on the device; :class:`EnsembleGraph` captures the lot in one
hipGraph, so a batch costs one graph launch.
"""
from __future__ import annotations

import os

import numpy as np
import torch
from torch import nn

from . import _lib, ops

MODALITIES = ("joint", "bone", "joint_motion", "bone_motion")   # inference_pipeline.py:25
ENSEMBLE_WEIGHTS_DEFAULT = (0.6, 0.6, 0.4, 0.4)                  # inference_pipeline.py:24

# (joint, parent), 0-indexed; joint 0 (NOSE) is its own parent (inference_pipeline.py:16-22)
MEDIAPIPE_BONE_PAIRS = (
    (0, 0), (1, 0), (2, 1), (3, 2), (4, 0), (5, 4), (6, 5), (7, 3), (8, 6), (9, 0), (10, 9),
    (11, 0), (12, 11), (13, 11), (14, 12), (15, 13), (16, 14), (17, 15), (18, 16), (19, 15),
    (20, 16), (21, 15), (22, 16), (23, 11), (24, 12), (25, 23), (26, 24), (27, 25), (28, 26),
    (29, 27), (30, 28), (31, 27), (32, 28))
# NTU RGB+D 25 joints, 1-indexed (v1, v2) of data_gen/gen_bone_data.py:4-16 -> 0-indexed;
# joint 21 (spine) is its own parent
NTU_BONE_PAIRS = tuple((a - 1, b - 1) for a, b in (
    (1, 2), (2, 21), (3, 21), (4, 3), (5, 21), (6, 5), (7, 6), (8, 7), (9, 21), (10, 9),
    (11, 10), (12, 11), (13, 1), (14, 13), (15, 14), (16, 15), (17, 1), (18, 17), (19, 18),
    (20, 19), (22, 23), (21, 21), (23, 8), (24, 25), (25, 12)))


def parent_table(bone_pairs, V):
    """(V,) int32 parent of each joint; every joint must appear exactly once."""
    par = np.full(V, -1, dtype=np.int32)
    for v, p in bone_pairs:
        if not (0 <= v < V and 0 <= p < V) or par[v] != -1:
            raise ValueError(f"bad bone pair ({v}, {p}) for V={V}")
        par[v] = p
    if (par < 0).any():
        raise ValueError("bone pairs do not cover every joint")
    return par


def derive_modalities(joint, parent, planes=False, data_bn=None, out=None):
    """All four streams of a joint batch ``(N, C, T, V, M)`` in one launch.

    ``planes=False``: returns four ``(N, C, T, V, M)`` tensors (derive_modalities' outputs,
    batched; bit-exact). ``planes=True``: four ``(N*M, C, T, V)`` tensors in the model's
    plane layout; with ``data_bn`` = (scale, shift), both ``(4, M*V*C)``, the models'
    eval-mode ``data_bn`` is applied as well (``Model.forward`` head, shift_gcn.py:194-198).
    """
    ops.check_input(joint, "joint")
    if joint.dim() != 5:
        raise ValueError("joint must be (N, C, T, V, M)")
    N, C, T, V, M = joint.shape
    if parent.dtype != torch.int32 or parent.numel() != V or parent.device != joint.device:
        raise ValueError("parent must be an int32 (V,) tensor on the joint's device")
    if out is None:
        shape = (N * M, C, T, V) if planes else (N, C, T, V, M)
        out = [torch.empty(shape, device=joint.device, dtype=torch.float32) for _ in range(4)]
    scale = shift = None
    if data_bn is not None:
        if not planes:
            raise ValueError("data_bn is applied in the plane layout only")
        scale, shift = data_bn
    with ops._timed("modalities", 0, 4 * joint.numel() * 5, joint):
        rc = _lib.load().sgcn_modalities(
            joint.data_ptr(), parent.data_ptr(), *[o.data_ptr() for o in out],
            None if scale is None else scale.data_ptr(),
            None if shift is None else shift.data_ptr(),
            int(planes), N, C, T, V, M, ops._stream(joint))
    _lib.check(rc, "sgcn_modalities")
    return out


# one stream per ensemble member (A/B knob: SGCN_ENS_STREAMS=0 runs them in order)
ENS_STREAMS = int(os.environ.get("SGCN_ENS_STREAMS", "1"))
_ENS_STREAMS = {}


def _ens_streams(device):
    s = _ENS_STREAMS.get(device)
    if s is None:
        s = _ENS_STREAMS[device] = [torch.cuda.Stream(device=device) for _ in range(4)]
    return s


class Ensemble(nn.Module):
    """``run_ensemble_inference`` over a batch: ``forward(joint)`` -> ``(scores, logits)``
    with ``scores`` = softmax(fused logits)[:, 1] (P(fall) for the MediaPipe models) and
    ``logits`` the float64 fused logits (N, num_class)."""

    def __init__(self, models, weights=ENSEMBLE_WEIGHTS_DEFAULT,
                 bone_pairs=MEDIAPIPE_BONE_PAIRS):
        super().__init__()
        if len(models) != 4 or len(weights) != 4:
            raise ValueError("one model and one weight per stream: " + ", ".join(MODALITIES))
        self.models = nn.ModuleList(models)
        self.weights = tuple(float(w) for w in weights)
        V = self.models[0].data_bn.num_features
        M = self.models[0].num_person
        self.num_point = V // (M * self.models[0].in_channels)
        self.register_buffer("parent", torch.from_numpy(
            parent_table(bone_pairs, self.num_point)), persistent=False)
        # alpha * logits is a float32 product in the reference (numpy float32 array times a
        # Python float), accumulated into a float64 zero vector in stream order
        self.register_buffer("alpha32", torch.tensor(self.weights, dtype=torch.float32),
                             persistent=False)

    def _data_bn_coef(self):
        """The four models' eval-mode data_bn coefficients, (4, F) each; computed once per
        version of those BatchNorms (ops.cached)."""
        bns = [m.data_bn for m in self.models]
        key = ops._src_key([t for bn in bns for t in (bn.weight, bn.bias, bn.running_mean,
                                                      bn.running_var)])
        key += tuple(float(bn.eps) for bn in bns)
        return ops.cached(self, "_sgcn_data_bn", key, self._make_data_bn_coef,
                          self.parent.device)

    def _make_data_bn_coef(self):
        F = self.models[0].data_bn.num_features
        dev = self.parent.device
        scale = torch.empty(4, F, device=dev, dtype=torch.float32)
        shift = torch.empty(4, F, device=dev, dtype=torch.float32)
        lib = _lib.load()
        for k, m in enumerate(self.models):
            bn = m.data_bn
            rc = lib.sgcn_bn_eval_coef(F, 0, bn.weight.data_ptr(), bn.bias.data_ptr(),
                                       bn.running_mean.data_ptr(), bn.running_var.data_ptr(),
                                       float(bn.eps), None, None, scale[k].data_ptr(),
                                       shift[k].data_ptr(), ops._stream(scale))
            _lib.check(rc, "sgcn_bn_eval_coef")
        return scale, shift

    @torch.no_grad()
    def forward(self, joint):
        if any(m.training for m in self.models):
            raise RuntimeError("Ensemble runs the models in eval mode (call .eval())")
        N, C, T, V, M = joint.shape
        streams = derive_modalities(joint, self.parent, planes=True,
                                    data_bn=self._data_bn_coef())
        acc = torch.zeros(N, self.models[0].fc.out_features, device=joint.device,
                          dtype=torch.float64)
        if ENS_STREAMS:
            # the four models are independent until the fused score: each runs on its own
            # stream (forked from and joined back into the current one; works inside a
            # hipGraph capture), so their MFMA- and HBM-bound phases overlap; the logits
            # are then accumulated in stream order as before
            cur = torch.cuda.current_stream(joint.device)
            subs = _ens_streams(joint.device)
            outs = []
            for m, xs, st in zip(self.models, streams, subs):
                st.wait_stream(cur)
                with torch.cuda.stream(st):
                    outs.append(m.forward_planes(xs, N, M))
                xs.record_stream(st)
            for st in subs:
                cur.wait_stream(st)
        else:
            outs = [m.forward_planes(xs, N, M) for m, xs in zip(self.models, streams)]
        for k, logits in enumerate(outs):
            acc = acc + (logits * self.alpha32[k]).double()
        # softmax exactly as inference_pipeline.py:364-365 (max-shifted exp in float64)
        e = torch.exp(acc - acc.max(dim=1, keepdim=True).values)
        scores = e[:, 1] / e.sum(dim=1)
        return scores, acc


# submodule (re)registrations anywhere: EnsembleGraph re-lists the ensemble's modules
_MODULE_EPOCH = [0]


def _module_registered(*_):
    _MODULE_EPOCH[0] += 1


torch.nn.modules.module.register_module_module_registration_hook(_module_registered)


def _state_key(mods):
    """Storage and version of every parameter and buffer of the modules ``mods`` (read
    from their own dicts, so a replaced parameter or buffer is seen; ~1 ms for the four
    MediaPipe models against ~4.7 ms through ``module.parameters()``)."""
    return [(t.data_ptr(), t._version) for m in mods for d in (m._parameters, m._buffers)
            for t in d.values() if t is not None]


class EnsembleGraph:
    """One hipGraph for a fixed batch shape: ``run(joint)`` copies the batch into the
    static input, replays the captured ensemble forward and returns (scores, logits)
    (views of static outputs, overwritten by the next ``run``).

    The eval-mode constants (BatchNorm coefficients, masks, folded conv+BatchNorm weights)
    are computed once per weight version outside the graph (ops.cached), so the graph holds
    the contraction and streaming kernels only; if any parameter or buffer of the ensemble
    has changed since the capture (an optimizer step, load_state_dict, a running-statistics
    update), ``run`` captures again first."""

    def __init__(self, ensemble: Ensemble, batch_shape, device):
        self.ensemble = ensemble
        self.device = device
        self.static_in = torch.zeros(batch_shape, device=device, dtype=torch.float32)
        self.captures = 0
        self._mods, self._epoch = list(ensemble.modules()), _MODULE_EPOCH[0]
        self._capture()

    def _capture(self):
        ensemble, device = self.ensemble, self.device
        self.graph = None
        side = torch.cuda.Stream(device)
        side.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(side):
            for _ in range(2):               # warm the caching allocator before capture
                ensemble(self.static_in)
        torch.cuda.current_stream(device).wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.scores, self.logits = ensemble(self.static_in)
        self.key = _state_key(self._mods)
        self.captures += 1

    def run(self, joint):
        if _MODULE_EPOCH[0] != self._epoch:   # a submodule was (re)registered somewhere
            self._mods, self._epoch = list(self.ensemble.modules()), _MODULE_EPOCH[0]
            self.key = None
        if _state_key(self._mods) != self.key:
            self._capture()
        self.static_in.copy_(joint, non_blocking=True)
        self.graph.replay()
        return self.scores, self.logits
