"""Shift_gcn's input gradient in one launch (round 6, verdict r05 next #5;
``sgcn_pw_fwd_gcn_dx``): the dX contraction of ``einsum('nwc,cd->nwd')`` (shift_gcn.py:131)
whose LDS-staged epilogue applies what ``sgcn_gcn_dx_finish`` did with the stored dXt — the
inverse shift_in rotation and the feature mask (shift_gcn.py:125-129), the residual-gradient
adds — and makes the mask-gradient and previous-bn2 backward partials per position tile.

* dx is bit-identical to sgcn_pw_fwd + sgcn_gcn_dx_finish (the same products and adds in the
  same order), for every operand combination the model uses, V = 25 / 33, ragged tiles;
* the partials sum (over tiles vs over planes) to the same totals within fp32 rounding, and
  through sgcn_mask_grad_finalize / sgcn_bn_bwd_finalize give the same gradients;
* in a training step the fused launch replaces every dX contraction + finish pair but l1's
  (3 input channels: no MFMA tile), and the model's gradients match the two-launch form.
"""
import numpy as np
import pytest
import torch

import formula

pytestmark = pytest.mark.gpu
DEV = "cuda"

CASES = [
    # (B, Cin, Cout, T, V)
    (3, 64, 64, 20, 25),
    (2, 64, 64, 300, 25),        # NTU plane length
    (2, 128, 128, 17, 25),       # P not a multiple of the 128-position tile
    (2, 256, 256, 9, 25),
    (2, 64, 128, 11, 33),        # MediaPipe joints
    (1, 128, 256, 7, 25),
    (2, 256, 128, 5, 33),
]


class _St:
    def __init__(self, mean, invstd):
        self.mean, self.invstd = mean, invstd


def _inputs(B, Cin, Cout, T, V, seed):
    g = torch.Generator().manual_seed(seed)
    r = lambda *s: torch.randn(*s, generator=g).to(DEV)
    w = r(Cin, Cout) / Cout ** 0.5
    dz = r(B, Cout, T, V)
    x0 = r(B, Cin, T, V)
    m = (torch.rand(1, V, Cin, generator=g) * 2).to(DEV)     # tanh(M) + 1 in (0, 2)
    add1, add2, add2m, ps = r(B, Cin, T, V), r(B, Cin, T, V), r(B, Cin, T, V), r(B, Cin, T, V)
    pst = _St(r(Cin), (torch.rand(Cin, generator=g) + 0.5).to(DEV))
    return w, dz, x0, m, add1, add2, add2m, ps, pst


@pytest.mark.parametrize("combo", ["identity_prev", "identity", "plain", "add1", "add2"])
@pytest.mark.parametrize("case", CASES, ids=["x".join(map(str, c)) for c in CASES])
def test_fused_matches_two_launch(case, combo):
    from shiftgcn import ops
    from shiftgcn.ops import PlaneView as PV
    B, Cin, Cout, T, V = case
    w, dz, x0, m, add1, add2, add2m, ps, pst = _inputs(*case, seed=sum(case) + len(combo))
    kw = {"identity_prev": dict(add1=add1, add2=add2, add2_mask=add2m, prev=(ps, pst)),
          "identity": dict(add1=add1, add2=add2, add2_mask=add2m),
          "plain": {}, "add1": dict(add1=add1), "add2": dict(add2=add2)}[combo]
    dxt = torch.empty(B, Cin, T, V, device=DEV)
    ops.pw_fwd(w, False, None, PV(dz), PV(dxt), Cin, Cout, T, V)
    ref = ops.gcn_dx_finish(dxt, x0, m, **kw)
    got = ops.gcn_dx_fused(w, dz, x0, m, **kw)
    torch.cuda.synchronize()
    # dx by torch (fp64 of the fp32 inputs): dXt[u] * m[u][c] (+ add1) (+ add2); the kernels
    # round dXt * m + add as one fma (as the finish kernel was compiled), so <= 1-2 ulp
    inv = (torch.arange(V, device=DEV)[None, :] - torch.arange(Cin, device=DEV)[:, None]) % V
    dxt_r = torch.gather(dxt.double(), 3, inv[None, :, None, :].expand(B, Cin, T, V))
    m_r = torch.gather(m[0].t().double(), 1, inv)[None, :, None, :]   # m[u][c] at (c, v')
    want = dxt_r * m_r
    if "add1" in kw:
        want = want + kw["add1"].double()
    if "add2" in kw:
        a2 = kw["add2"].double()
        want = want + (torch.where(kw["add2_mask"] > 0, a2, torch.zeros_like(a2))
                       if "add2_mask" in kw else a2)
    assert torch.allclose(got[0].double(), want, rtol=3e-7, atol=1e-7 * float(want.abs().max()))
    assert torch.equal(got[0], ref[0])            # dx, bit for bit
    rows = got[2]
    assert rows == -(-(B * T * V) // (256 if Cin <= 64 else 128))
    # mask-gradient partials: per tile vs per plane, the same totals per (c, u)
    s_ref = ref[1].double().view(B, Cin, V).sum(0)
    s_got = got[1].double().view(rows, Cin, V).sum(0)
    # (an independent fp64 total: sum over (b, t) of dXt[u] * x0[(u + c) mod V])
    d64, x64 = dxt.double(), x0.double()
    idx = (torch.arange(V, device=DEV)[None, :] + torch.arange(Cin, device=DEV)[:, None]) % V
    xr = torch.gather(x64, 3, idx[None, :, None, :].expand(B, Cin, T, V))
    want = (d64 * xr).sum((0, 2))
    scale = float(want.abs().max())
    assert float((s_got - want).abs().max()) <= 2e-6 * scale * (T * B) ** 0.5
    assert float((s_ref - want).abs().max()) <= 2e-6 * scale * (T * B) ** 0.5
    if combo == "identity_prev":
        p_ref = ref[2].double().view(B, Cin, 2).sum(0)
        p_got = got[3].double().view(rows, Cin, 2).sum(0)
        tol = 2e-6 * float(p_ref.abs().max()) * (T * B) ** 0.5
        assert float((p_got - p_ref).abs().max()) <= tol
        # and through the finalizes the model uses
        mref = ops.mask_grad_finalize(ref[1], m, B, Cin, V)
        mgot = ops.mask_grad_finalize(got[1], m, rows, Cin, V)
        torch.cuda.synchronize()
        assert torch.allclose(mgot, mref, rtol=1e-5, atol=1e-6 * float(mref.abs().max()))


def _model_grads(fused_dx, monkeypatch, steps=1):
    import shiftgcn
    from shiftgcn import fused
    monkeypatch.setattr(fused, "GCN_DX_FUSED", fused_dx)
    m = shiftgcn.Model(num_class=10, num_point=25, num_person=2, graph="graph.ntu_rgb_d.Graph")
    formula.fill_state(m, seed=12)
    m = m.to(DEV).train()
    x = formula.tensor((4, 3, 64, 25, 2), 90, 1.0).to(DEV)
    y = torch.tensor([1, 2, 3, 4], device=DEV)
    loss = torch.nn.functional.cross_entropy(m(x), y)
    loss.backward()
    torch.cuda.synchronize()
    return {n: p.grad.detach().double().cpu() for n, p in m.named_parameters()
            if p.grad is not None}


def test_model_gradients_match_two_launch(monkeypatch):
    """The whole model: every gradient within fp32 summation-order noise of the two-launch
    form (the dx tensors are identical; only the mask-gradient and bn2 partial sums change
    order), and the fused launch is what runs (9 of the 10 units: l1 has 3 input channels)."""
    from shiftgcn import ops
    calls = {"fused": 0, "finish": 0}
    real_f, real_n = ops.gcn_dx_fused, ops.gcn_dx_finish

    def spy_f(*a, **k):
        calls["fused"] += 1
        return real_f(*a, **k)

    def spy_n(*a, **k):
        calls["finish"] += 1
        return real_n(*a, **k)

    monkeypatch.setattr(ops, "gcn_dx_fused", spy_f)
    monkeypatch.setattr(ops, "gcn_dx_finish", spy_n)
    got = _model_grads(1, monkeypatch)
    assert calls == {"fused": 9, "finish": 1}, calls   # (with the knob on)
    ref = _model_grads(0, monkeypatch)
    assert got.keys() == ref.keys() and len(got) > 100
    flips = 0
    for n in ref:
        if n.endswith("pos"):   # sign-normalised +-0.01 (.cu:370-395): a near-zero plane sum
            flips += int((got[n] != ref[n]).sum())   # may change sign with the order
            continue
        if n.endswith(("gcn1.Linear_bias", "down.0.bias", "residual.conv.bias")):
            # a bias right before a training BatchNorm has an exactly zero gradient (the
            # batch mean removes it): both values are rounding residue of sum(dZ) = 0, so
            # bound them against the layer's weight gradient instead
            wn = n[:-len("bias")] + ("weight" if n.endswith(".bias") else "")
            wn = wn.replace("Linear_", "Linear_weight") if n.endswith("Linear_bias") else wn
            wscale = float(ref[wn].abs().max())
            assert float((got[n] - ref[n]).abs().max()) <= 1e-3 * wscale, n
            continue
        scale = float(ref[n].abs().max())
        if scale == 0.0:
            assert float(got[n].abs().max()) == 0.0, n
            continue
        err = float((got[n] - ref[n]).abs().max()) / scale
        # (BatchNorm gradients amplify summation-order differences through 10 units)
        assert err <= 2e-4, (n, err)
    assert flips <= 1, flips
