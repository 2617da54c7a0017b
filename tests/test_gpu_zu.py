"""Shift_gcn's shift_out applied by the BatchNorm kernels' addressing (per_joint = 3,
shift_gcn.py:114-118,136) instead of by the contraction's rotated stores: every kernel on
the pre-rotation tensor equals the per_joint = 1/2 kernel on the rotated tensor (bit for
bit where the arithmetic order is the same; the apply pass's output moments up to
summation order)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
CASES = [(3, 64, 20, 25), (2, 128, 9, 25), (2, 48, 11, 33)]


def _rot(zu):
    """logical z[c, t, w] = zu[c, t, (w - c) mod V]"""
    B, C, T, V = zu.shape
    idx = (torch.arange(V, device=zu.device)[None, :] - torch.arange(C, device=zu.device)[:, None]) % V
    return zu.gather(3, idx.view(1, C, 1, V).expand(B, C, T, V))


@pytest.mark.parametrize("case", CASES, ids=["x".join(map(str, c)) for c in CASES])
def test_zu_kernels_match_rotated(case):
    from shiftgcn import ops
    import torch.nn as nn
    B, C, T, V = case
    g = torch.Generator().manual_seed(sum(case))
    zu = (torch.randn(B, C, T, V, generator=g) * 2 + 0.3).to(DEV)
    zr = _rot(zu)
    res = torch.randn(B, C, T, V, generator=g).to(DEV)
    bn = nn.BatchNorm1d(C * V).to(DEV)
    with torch.no_grad():
        bn.weight.copy_(torch.rand(C * V, generator=g) + 0.5)
        bn.bias.copy_(torch.randn(C * V, generator=g))
    p1, p3 = ops.moments(zr, 1), ops.moments(zu, 3)
    torch.cuda.synchronize()
    assert torch.equal(p1, p3)
    st = ops.bn_finalize(p1, B, C * V, T, bn, perm_V=V)
    h1, s1 = ops.bn_apply(zr, st, 1, r=res, relu=True, out_stats=True)
    h3, s3 = ops.bn_apply(zu, st, 3, r=res, relu=True, out_stats=True)
    torch.cuda.synchronize()
    assert torch.equal(h1, h3)
    assert float((s1 - s3).abs().max()) <= 1e-5 * float(s1.abs().max())
    dA = torch.randn(B, C, T, V, generator=g).to(DEV)
    coef = torch.randn(3, C, generator=g).to(DEV)
    r1, _ = ops.bn_bwd_reduce(dA, h1, True, zr, st, 1, dy_coef=coef)
    r3, _ = ops.bn_bwd_reduce(dA, h1, True, zu, st, 3, dy_coef=coef)
    torch.cuda.synchronize()
    assert torch.equal(r1, r3)
    cz, _, _ = ops.bn_bwd_finalize(r1, B, C * V, B * T, st, bn, perm_V=V)
    gi1 = torch.empty_like(dA)
    gi3 = torch.empty_like(dA)
    d1 = ops.bn_bwd_apply(dA, h1, True, zr, cz, 2, dr=gi1, dy_coef=coef)
    d3 = ops.bn_bwd_apply(dA, h1, True, zu, cz, 3, dr=gi3, dy_coef=coef)
    torch.cuda.synchronize()
    assert torch.equal(d1, d3) and torch.equal(gi1, gi3)


def test_unit_parity_zu_off(monkeypatch):
    """The rotated-store form (SGCN_GCN_ZU=0) keeps unit parity with the oracle."""
    import formula
    import shiftgcn
    from oracle import model_oracle as mo
    from shiftgcn import fused
    from test_gpu_blocks import _compare
    monkeypatch.setattr(fused, "GCN_ZU", 0)
    ref = mo.TCN_GCN_unit(64, 128, None, stride=2, num_point=25)
    formula.fill_state(ref, seed=29)
    ours = shiftgcn.TCN_GCN_unit(64, 128, None, stride=2, num_point=25).to(DEV)
    ours.load_state_dict(ref.state_dict())
    x = formula.tensor((3, 64, 14, 25), 81, 1.0)
    g = formula.tensor((3, 128, 7, 25), 82, 1.0)
    xr = x.clone().requires_grad_(True)
    yr = ref(xr)
    yr.backward(g)
    xo = x.to(DEV).requires_grad_(True)
    yo = ours(xo)
    yo.backward(g.to(DEV))
    torch.cuda.synchronize()
    _compare(ref, ours, xr, yr, xo, yo, "zu-off")
