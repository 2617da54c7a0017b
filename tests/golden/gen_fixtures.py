"""Generate the committed golden fixtures by running the REFERENCE Python code on CPU.

Run only where ``/root/reference`` exists (this build container):

    python tests/golden/gen_fixtures.py

What runs: the reference's own ``model/shift_gcn.py`` modules and its
``model/Temporal_shift/cuda/shift.py`` autograd glue (imported from
``/root/reference``), with the reference CUDA extension ``shift_cuda`` — which cannot be
built or run here — replaced by a module whose ``forward``/``backward`` call the numpy
restatement :mod:`oracle.shift_oracle` of ``shift_cuda_kernel.cu``. ``torch.zeros`` /
``torch.ones`` drop ``device='cuda'`` during construction (the CPU recipe the reference
documents at ``CLAUDE.md:33``). Weights and inputs come from ``formula.py``; only
outputs are stored. Nothing from the reference source is copied into the fixtures.

Output: ``tests/golden/*.npz`` (small; read by ``tests/test_oracle_*.py`` and the GPU
parity tests on the GPU box, where ``/root/reference`` does not exist).
"""
from __future__ import annotations

import contextlib
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from oracle import shift_oracle as so  # noqa: E402
import formula  # noqa: E402


def _install_shift_cuda():
    mod = types.ModuleType("shift_cuda")

    def forward(inp, xpos, ypos, stride):
        out = so.shift_forward(inp.detach().numpy(), xpos.detach().numpy(),
                               ypos.detach().numpy(), stride)
        return torch.from_numpy(out)

    def backward(gout, inp, out, xpos, ypos, stride):
        gin, gx, gy = so.shift_backward(gout.detach().numpy(), inp.detach().numpy(),
                                        xpos.detach().numpy(), ypos.detach().numpy(), stride)
        return [torch.from_numpy(gin), torch.from_numpy(gx), torch.from_numpy(gy)]

    mod.forward, mod.backward = forward, backward
    sys.modules["shift_cuda"] = mod


@contextlib.contextmanager
def _cpu_construction():
    z0, o0 = torch.zeros, torch.ones

    def strip(fn):
        def inner(*a, **k):
            k.pop("device", None)
            return fn(*a, **k)
        return inner

    torch.zeros, torch.ones = strip(z0), strip(o0)
    try:
        yield
    finally:
        torch.zeros, torch.ones = z0, o0


def _import_reference():
    _install_shift_cuda()
    for p in (REF, os.path.join(REF, "model", "Temporal_shift")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import model.shift_gcn as ref_sg  # noqa: E402
    from cuda import shift as ref_shift  # noqa: E402
    return ref_sg, ref_shift


def _np(t):
    return t.detach().cpu().numpy().copy()


def gen_indices(ref_sg, out):
    """Fixture 1: spatial shift index arrays (shift_gcn.py:108-118), bit-exact int64."""
    with _cpu_construction():
        for V in (25, 33):
            for C in (3, 64, 128, 256):
                g = ref_sg.Shift_gcn(C, C, None, num_point=V)
                out[f"shift_in_V{V}_C{C}"] = _np(g.shift_in)
                out[f"shift_out_V{V}_C{C}"] = _np(g.shift_out)


SHIFT_CASES = [
    # (name, B, C, H, W, stride)
    ("s1", 2, 8, 20, 25, 1),
    ("s2", 2, 8, 20, 25, 2),
    ("s2odd", 2, 8, 21, 25, 2),
    ("s1v33", 1, 6, 12, 33, 1),
]


def shift_case_inputs(name, B, C, H, W, stride):
    """Inputs of a Shift fixture case (also rebuilt by the tests)."""
    k = sum(map(ord, name))
    x = formula.tensor((B, C, H, W), 11 + k, 1.0)
    g = formula.tensor((B, C, H // stride, W), 13 + k, 1.0)
    xpos = formula.tensor((C,), 17 + k, 1e-8)
    ypos = formula.tensor((C,), 19 + k, 3.0)
    # exercise the edge cases: exact integers, zero, |y| > H, x = +-1e-8 and 0, and x
    # beyond the joint axis
    ypos[0], ypos[1], ypos[2] = 0.0, 2.0, -1.0
    ypos[3] = float(H + 3)
    xpos[0], xpos[1], xpos[2] = 0.0, 1e-8, -1e-8
    xpos[3] = 1.25
    xpos[4] = -2.5
    return x, g, xpos, ypos


def gen_shift(ref_shift, out):
    """Fixture 2: Shift fwd/bwd through the reference ShiftFunction glue (shift.py:9-30)."""
    for name, B, C, H, W, stride in SHIFT_CASES:
        x, g, xpos, ypos = shift_case_inputs(name, B, C, H, W, stride)
        xr = x.clone().requires_grad_(True)
        xp = xpos.clone().requires_grad_(True)
        yp = ypos.clone().requires_grad_(True)
        y = ref_shift.ShiftFunction.apply(xr, xp, yp, stride)
        y.backward(g)
        out[f"shift_{name}_out"] = _np(y)
        out[f"shift_{name}_gin"] = _np(xr.grad)
        out[f"shift_{name}_gx"] = _np(xp.grad)
        out[f"shift_{name}_gy"] = _np(yp.grad)


BLOCK_CASES = [
    # (name, kind, Cin, Cout, NM, T, V, stride)
    ("gcn_3_16", "gcn", 3, 16, 4, 6, 25, 1),
    ("gcn_16_32", "gcn", 16, 32, 4, 8, 25, 1),
    ("gcn_32_32", "gcn", 32, 32, 3, 6, 33, 1),
    ("tcn_16_s1", "tcn", 16, 16, 4, 8, 25, 1),
    ("tcn_16_s2", "tcn", 16, 16, 4, 10, 25, 2),
    ("unit_8_16_s2", "unit", 8, 16, 4, 10, 25, 2),
    ("unit_16_16_s1", "unit", 16, 16, 3, 8, 25, 1),
    ("unit_3_16_nores", "unit_nores", 3, 16, 2, 6, 25, 1),
]


def build_block(mods, kind, cin, cout, V, stride):
    if kind == "gcn":
        return mods.Shift_gcn(cin, cout, None, num_point=V)
    if kind == "tcn":
        return mods.Shift_tcn(cin, cout, stride=stride)
    if kind == "unit":
        return mods.TCN_GCN_unit(cin, cout, None, stride=stride, num_point=V)
    if kind == "unit_nores":
        return mods.TCN_GCN_unit(cin, cout, None, stride=stride, residual=False, num_point=V)
    raise ValueError(kind)


def block_case_inputs(name, kind, cin, cout, NM, T, V, stride):
    k = sum(map(ord, name))
    x = formula.tensor((NM, cin, T, V), 23 + k, 1.0)
    To = T // stride if kind != "gcn" else T
    g = formula.tensor((NM, cout, To, V), 29 + k, 1.0)
    return x, g


def gen_blocks(ref_sg, out):
    """Fixture 3/4: Shift_gcn, Shift_tcn, TCN_GCN_unit fwd + every grad, train-mode BN."""
    for name, kind, cin, cout, NM, T, V, stride in BLOCK_CASES:
        with _cpu_construction():
            m = build_block(ref_sg, kind, cin, cout, V, stride)
        formula.fill_state(m, seed=31 + sum(map(ord, name)))
        m.train()
        x, g = block_case_inputs(name, kind, cin, cout, NM, T, V, stride)
        xr = x.clone().requires_grad_(True)
        y = m(xr)
        y.backward(g)
        out[f"blk_{name}_out"] = _np(y)
        out[f"blk_{name}_gx"] = _np(xr.grad)
        for pn, p in m.named_parameters():
            if p.grad is not None:
                out[f"blk_{name}_grad.{pn}"] = _np(p.grad)
        for bn, b in m.named_buffers():
            if b.dtype.is_floating_point:
                out[f"blk_{name}_buf.{bn}"] = _np(b)


MODEL_CASES = [
    # (name, num_class, V, M, N, T)
    ("ntu", 60, 25, 2, 2, 300),
    ("mp", 2, 33, 1, 2, 300),
]


def model_case_inputs(name, num_class, V, M, N, T):
    k = sum(map(ord, name))
    x = formula.tensor((N, 3, T, V, M), 41 + k, 1.0)
    labels = torch.from_numpy(
        (np.abs(formula.hash_uniform(N, 43 + k)) * 2 * num_class).astype(np.int64) % num_class)
    return x, labels


def gen_models(ref_sg, out):
    """Fixture 5/6: Model logits (train and eval), loss, grad checksums, one SGD step."""
    graph_mod = types.ModuleType("fixture_graph")

    class Graph:  # the graph object's adjacency is never used by the compute path
        def __init__(self, **kw):
            self.A = np.zeros((3, 1, 1))

    graph_mod.Graph = Graph
    sys.modules["fixture_graph"] = graph_mod
    for name, num_class, V, M, N, T in MODEL_CASES:
        with _cpu_construction():
            m = ref_sg.Model(num_class=num_class, num_point=V, num_person=M,
                             graph="fixture_graph.Graph")
        formula.fill_state(m, seed=97 + sum(map(ord, name)))
        x, labels = model_case_inputs(name, num_class, V, M, N, T)
        m.eval()
        with torch.no_grad():
            out[f"model_{name}_logits_eval"] = _np(m(x))
        m.train()
        logits = m(x)
        loss = torch.nn.functional.cross_entropy(logits, labels)
        loss.backward()
        out[f"model_{name}_logits_train"] = _np(logits)
        out[f"model_{name}_loss"] = _np(loss)
        names, gsum, gnorm = [], [], []
        for pn, p in m.named_parameters():
            if p.grad is None:
                continue
            names.append(pn)
            gsum.append(float(p.grad.double().sum()))
            gnorm.append(float(p.grad.double().norm()))
            if pn.endswith(("xpos", "ypos")) or p.numel() <= 512:
                out[f"model_{name}_grad.{pn}"] = _np(p.grad)
        out[f"model_{name}_grad_names"] = np.array(names)
        out[f"model_{name}_grad_sum"] = np.array(gsum)
        out[f"model_{name}_grad_norm"] = np.array(gnorm)
        # one SGD step with the reference parameter groups (main.py:301-322)
        groups = []
        for key, value in m.named_parameters():
            wd = 1e-4
            if "Linear_weight" in key:
                wd = 1e-3
            elif "Mask" in key:
                wd = 0.0
            groups.append({"params": value, "lr": 0.1, "weight_decay": wd})
        opt = torch.optim.SGD(groups, momentum=0.9, nesterov=True)
        opt.step()
        out[f"model_{name}_step_param_sum"] = np.array(
            [float(p.detach().double().sum()) for pn, p in m.named_parameters()
             if p.dtype.is_floating_point])
        # the same forward/backward in float64 (conditioning reference: model-level fp32
        # gradients through 10 BN units at bs=2 differ from it by up to ~3e-3 even on the
        # reference's own fp32 path)
        with _cpu_construction():
            m64 = ref_sg.Model(num_class=num_class, num_point=V, num_person=M,
                               graph="fixture_graph.Graph")
        formula.fill_state(m64, seed=97 + sum(map(ord, name)))
        m64 = m64.double().train()
        logits64 = m64(x.double())
        torch.nn.functional.cross_entropy(logits64, labels).backward()
        out[f"model_{name}_logits_train64"] = _np(logits64)
        p64 = dict(m64.named_parameters())
        out[f"model_{name}_grad_norm64"] = np.array([float(p64[n].grad.norm()) for n in names])
        out[f"model_{name}_grad_sum64"] = np.array([float(p64[n].grad.sum()) for n in names])
        for n in names:
            if n.endswith(("xpos", "ypos")):
                out[f"model_{name}_grad64.{n}"] = _np(p64[n].grad)
        # ... and its SGD step: the fp32 step's own deviation from it (per parameter sum)
        # is the bar the HIP step is held to (tests/test_train_step.py)
        groups64 = []
        for key, value in m64.named_parameters():
            wd = 1e-4
            if "Linear_weight" in key:
                wd = 1e-3
            elif "Mask" in key:
                wd = 0.0
            groups64.append({"params": value, "lr": 0.1, "weight_decay": wd})
        torch.optim.SGD(groups64, momentum=0.9, nesterov=True).step()
        out[f"model_{name}_step_param_sum64"] = np.array(
            [float(p.detach().sum()) for pn, p in m64.named_parameters()
             if p.dtype.is_floating_point])


def main():
    torch.set_num_threads(max(1, os.cpu_count() or 1))
    ref_sg, ref_shift = _import_reference()
    out = {}
    gen_indices(ref_sg, out)
    gen_shift(ref_shift, out)
    np.savez_compressed(os.path.join(HERE, "shift_fixtures.npz"), **out)
    out = {}
    gen_blocks(ref_sg, out)
    np.savez_compressed(os.path.join(HERE, "block_fixtures.npz"), **out)
    out = {}
    gen_models(ref_sg, out)
    np.savez_compressed(os.path.join(HERE, "model_fixtures.npz"), **out)
    for f in ("shift_fixtures.npz", "block_fixtures.npz", "model_fixtures.npz"):
        print(f, os.path.getsize(os.path.join(HERE, f)), "bytes")


if __name__ == "__main__":
    main()
