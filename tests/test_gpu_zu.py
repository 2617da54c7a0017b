"""Shift_gcn.bn on the contraction output stored BEFORE its shift_out (per_joint = 3,
shift_gcn.py:114-118,136-137): the BatchNorm kernels apply the joint rotation in their
addressing. Each kernel is checked against an fp64 torch evaluation on the logical
(rotated) tensor z[c, t, w] = zu[c, t, (w - c) mod V]: statistics, apply (+ residual, ReLU,
output moments), backward partials with the on-the-fly input gradient, and the backward
apply whose dZ is stored back in the pre-rotation layout."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
CASES = [(3, 64, 20, 25), (2, 128, 9, 25), (2, 48, 11, 33)]


def _idx(C, V, dev):
    return (torch.arange(V, device=dev)[None, :] - torch.arange(C, device=dev)[:, None]) % V


def _rot(zu):
    """logical z[c, t, w] = zu[c, t, (w - c) mod V]"""
    B, C, T, V = zu.shape
    return zu.gather(3, _idx(C, V, zu.device).view(1, C, 1, V).expand(B, C, T, V))


def _close(a, b, tol):
    a, b = a.double(), b.double()
    return float((a - b).abs().max()) <= tol * (float(b.abs().max()) + 1e-30)


@pytest.mark.parametrize("case", CASES, ids=["x".join(map(str, c)) for c in CASES])
def test_zu_kernels_match_torch(case):
    from shiftgcn import ops
    import torch.nn as nn
    B, C, T, V = case
    g = torch.Generator().manual_seed(sum(case))
    zu = (torch.randn(B, C, T, V, generator=g) * 2 + 0.3).to(DEV)
    z = _rot(zu).double()
    res = torch.randn(B, C, T, V, generator=g).to(DEV)
    bn = nn.BatchNorm1d(C * V).to(DEV)
    with torch.no_grad():
        bn.weight.copy_(torch.rand(C * V, generator=g) + 0.5)
        bn.bias.copy_(torch.randn(C * V, generator=g))
    # statistics (local feature f = c*V + w; the module's feature is w*C + c)
    st = ops.bn_finalize(ops.moments(zu, 3), B, C * V, T, bn, perm_V=V)
    mean = z.mean((0, 2))                                   # (C, V)
    var = z.var((0, 2), unbiased=False)
    torch.cuda.synchronize()
    assert _close(st.mean.view(C, V), mean, 1e-6)
    assert _close(st.invstd.view(C, V), (var + bn.eps).rsqrt(), 1e-6)
    # apply + residual + ReLU, with the output's per-plane moments
    sc, sh = st.scale.double().view(1, C, 1, V), st.shift.double().view(1, C, 1, V)
    h_ref = torch.relu(z * sc + sh + res.double())
    h, hs = ops.bn_apply(zu, st, 3, r=res, relu=True, out_stats=True)
    torch.cuda.synchronize()
    assert _close(h, h_ref, 1e-6)
    hs = hs.view(B * C, 2).double()
    assert _close(hs[:, 0], h_ref.mean((2, 3)).flatten(), 1e-5)
    assert _close(hs[:, 1], h_ref.var((2, 3), unbiased=False).flatten() * T * V, 1e-5)
    # backward partials with dy = k1*dA + k2*h + k3 (the following BatchNorm's dx)
    dA = torch.randn(B, C, T, V, generator=g).to(DEV)
    coef = torch.randn(3, C, generator=g).to(DEV)
    part, _ = ops.bn_bwd_reduce(dA, h, True, zu, st, 3, dy_coef=coef)
    k = coef.double().view(3, 1, C, 1, 1)
    gd = (k[0] * dA.double() + k[1] * h.double() + k[2]) * (h > 0)
    xhat = (z - mean.view(1, C, 1, V)) * st.invstd.double().view(1, C, 1, V)
    p = part.view(B, C, V, 2).double()
    torch.cuda.synchronize()
    assert _close(p[..., 0], gd.sum(2), 1e-5)
    assert _close(p[..., 1], (gd * xhat).sum(2), 1e-5)
    # backward apply: dZ at the pre-rotation position, identity-residual gradient = g
    cz, _, _ = ops.bn_bwd_finalize(part, B, C * V, B * T, st, bn, perm_V=V)
    gi = torch.empty_like(dA)
    dz = ops.bn_bwd_apply(dA, h, True, zu, cz, 3, dr=gi, dy_coef=coef)
    c = cz.double().view(3, 1, C, 1, V)
    dz_ref = c[0] * gd + c[1] * z + c[2]
    torch.cuda.synchronize()
    assert _close(_rot(dz), dz_ref, 1e-5)
    assert _close(gi, gd, 1e-6)


def test_rejected_layouts_refused():
    """per_joint 1 / 2 (the rotated-store layouts, ABI <= 18) are gone: SGCN_EINVAL."""
    from shiftgcn import ops
    x = torch.randn(2, 8, 4, 25, device=DEV)
    for pj in (1, 2):
        with pytest.raises(ValueError, match="invalid argument"):
            ops.moments(x, pj)
