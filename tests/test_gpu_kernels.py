"""GPU: MFMA pointwise-contraction and BatchNorm kernels vs plain PyTorch fp64 references
(including the fused joint-shift rotations, feature mask, time stride, ReLU, accumulate)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rot_gather(x, sign):
    """x[b, c, t, (v + sign*c) mod V] (the shift_in-style gather of a plane operand)."""
    B, C, T, V = x.shape
    v = torch.arange(V, device=x.device)
    c = torch.arange(C, device=x.device)
    idx = (v[None, :] + sign * c[:, None]) % V                 # (C, V)
    return torch.gather(x, 3, idx[None, :, None, :].expand(B, C, T, V))


def rot_scatter(y, sign):
    """out[b, m, t, (v + sign*m) mod V] = y[b, m, t, v]."""
    B, M, T, V = y.shape
    v = torch.arange(V, device=y.device)
    m = torch.arange(M, device=y.device)
    idx = (v[None, :] + sign * m[:, None]) % V
    out = torch.empty_like(y)
    out.scatter_(3, idx[None, :, None, :].expand(B, M, T, V), y)
    return out


@pytest.mark.parametrize("M,K", [(64, 3), (64, 64), (128, 64), (128, 128), (256, 128),
                                 (256, 256), (3, 64), (64, 256), (100, 37), (37, 51), (17, 64),
                                 (4, 130), (1, 7)])
@pytest.mark.parametrize("rin,rout,mask", [(0, 0, False), (1, 1, True), (1, 0, False)])
def test_pw_fwd_matches_torch(M, K, rin, rout, mask):
    from shiftgcn import ops
    torch.manual_seed(M * 7 + K)
    B, T, V = 3, 13, 25
    x = torch.randn(B, K, T, V, device=DEV)
    w = torch.randn(M, K, device=DEV) / K ** 0.5
    bias = torch.randn(M, device=DEV)
    mk = (torch.rand(V, K, device=DEV) + 0.5) if mask else None
    y = torch.empty(B, M, T, V, device=DEV)
    ops.pw_fwd(w, False, bias, ops.PlaneView(x, 1, rin), ops.PlaneView(y, 1, rout), M, K, T, V,
               mask=mk, relu=True)
    xg = rot_gather(x.double(), rin) if rin else x.double()
    if mask:
        xg = xg * mk.double().t()[None, :, None, :]
    ref = torch.einsum("mk,bktv->bmtv", w.double(), xg) + bias.double()[None, :, None, None]
    ref = torch.relu(ref)
    if rout:
        ref = rot_scatter(ref, rout)
    torch.testing.assert_close(y.double(), ref, rtol=1e-5, atol=1e-5)
    # m-contiguous weights (Linear_weight layout) + accumulate
    y2 = y.clone()
    ops.pw_fwd(w.t().contiguous(), True, bias, ops.PlaneView(x, 1, rin),
               ops.PlaneView(y2, 1, rout), M, K, T, V, mask=mk, relu=True, accumulate=True)
    torch.testing.assert_close(y2.double(), 2 * ref, rtol=1e-5, atol=2e-5)


@pytest.mark.parametrize("M", [128, 64])
def test_pw_fwd_time_stride(M):
    """(M = 64: the streaming contraction for M, K <= 64, both directions)"""
    from shiftgcn import ops
    torch.manual_seed(3)
    B, K, T, V = 2, 64, 21, 25
    To = (T - 1) // 2 + 1
    x = torch.randn(B, K, T, V, device=DEV)
    w = torch.randn(M, K, device=DEV) / 8
    y = torch.empty(B, M, To, V, device=DEV)
    ops.pw_fwd(w, False, None, ops.PlaneView(x, 2), ops.PlaneView(y), M, K, To, V)
    ref = torch.einsum("mk,bktv->bmtv", w.double(), x.double()[:, :, ::2])
    torch.testing.assert_close(y.double(), ref, rtol=1e-5, atol=1e-5)
    # transposed (dX) with strided output rows, accumulating
    dx = torch.zeros(B, K, T, V, device=DEV)
    g = torch.randn(B, M, To, V, device=DEV)
    ops.pw_fwd(w, True, None, ops.PlaneView(g), ops.PlaneView(dx, 2), K, M, To, V,
               accumulate=True)
    ref = torch.zeros(B, K, T, V, dtype=torch.float64, device=DEV)
    ref[:, :, ::2] = torch.einsum("mk,bmtv->bktv", w.double(), g.double())
    torch.testing.assert_close(dx.double(), ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("M,Nc", [(64, 3), (64, 64), (128, 64), (128, 128), (256, 256),
                                  (64, 128), (37, 100), (64, 1), (100, 2), (17, 4)])
@pytest.mark.parametrize("grot,xrot,mask,transpose", [(0, 0, False, False),
                                                       (1, 1, True, True)])
def test_pw_dw_matches_torch(M, Nc, grot, xrot, mask, transpose):
    from shiftgcn import ops
    torch.manual_seed(M + Nc)
    B, T, V = 4, 17, 25
    gr = torch.randn(B, M, T, V, device=DEV)
    x = torch.randn(B, Nc, T, V, device=DEV)
    mk = (torch.rand(V, Nc, device=DEV) + 0.5) if mask else None
    dw = torch.empty((Nc, M) if transpose else (M, Nc), device=DEV)
    db = torch.empty(M, device=DEV)
    ops.pw_dw(ops.PlaneView(gr, 1, grot), ops.PlaneView(x, 1, xrot), dw, M, Nc, T, V, mask=mk,
              transpose=transpose, dbias=db)
    G = rot_gather(gr.double(), grot) if grot else gr.double()
    X = rot_gather(x.double(), xrot) if xrot else x.double()
    if mask:
        X = X * mk.double().t()[None, :, None, :]
    ref = torch.einsum("bmtv,bctv->mc", G, X)
    if transpose:
        ref = ref.t()
    torch.testing.assert_close(dw.double(), ref, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(db.double(), G.sum((0, 2, 3)), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("B,T,V,Nc", [(3, 1, 5, 128), (2, 9, 33, 128), (5, 7, 25, 200)])
def test_pw_dw_strided_and_tiny_planes(B, T, V, Nc):
    """Wide contractions (the pw_dw3 path): a temporal-stride-2 X view, samples smaller than
    one position chunk (T*V < 16), V=33 rotations, ragged channel counts."""
    from shiftgcn import ops
    torch.manual_seed(B * 100 + T)
    M = 128
    To = T
    Ti = 2 * T
    gr = torch.randn(B, M, To, V, device=DEV)
    x = torch.randn(B, Nc, Ti, V, device=DEV)
    mk = torch.rand(V, Nc, device=DEV) + 0.5
    dw = torch.empty(M, Nc, device=DEV)
    db = torch.empty(M, device=DEV)
    ops.pw_dw(ops.PlaneView(gr, 1, -1), ops.PlaneView(x, 2, 1), dw, M, Nc, To, V, mask=mk,
              dbias=db)
    G = rot_gather(gr.double(), -1)
    X = rot_gather(x.double()[:, :, ::2], 1) * mk.double().t()[None, :, None, :]
    torch.testing.assert_close(dw.double(), torch.einsum("bmtv,bctv->mc", G, X),
                               rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(db.double(), G.sum((0, 2, 3)), rtol=1e-5, atol=1e-4)


def test_pw_dw_large_split_is_deterministic():
    from shiftgcn import ops
    torch.manual_seed(0)
    B, M, Nc, T, V = 32, 256, 256, 75, 25
    gr = torch.randn(B, M, T, V, device=DEV)
    x = torch.randn(B, Nc, T, V, device=DEV)
    a = torch.empty(M, Nc, device=DEV)
    b = torch.empty(M, Nc, device=DEV)
    ops.pw_dw(ops.PlaneView(gr), ops.PlaneView(x), a, M, Nc, T, V)
    ops.pw_dw(ops.PlaneView(gr), ops.PlaneView(x), b, M, Nc, T, V)
    assert torch.equal(a, b)
    ref = torch.einsum("bmtv,bctv->mc", gr.double(), x.double())
    torch.testing.assert_close(a.double(), ref, rtol=1e-5, atol=2e-3)


def _rot(zu):
    """logical z[c, t, w] = zu[c, t, (w - c) mod V] (Shift_gcn's shift_out,
    shift_gcn.py:114-118,136)"""
    B, C, T, V = zu.shape
    idx = (torch.arange(V, device=zu.device)[None, :] - torch.arange(C, device=zu.device)[:, None]) % V
    return zu.gather(3, idx.view(1, C, 1, V).expand(B, C, T, V))


@pytest.mark.parametrize("per_joint", [False, True])
def test_bn_train_forward_backward_matches_torch(per_joint):
    """per_joint: Shift_gcn.bn (BatchNorm1d over (b, t) of (v, c) features) on the
    contraction output stored before its shift_out (per_joint = 3: the kernels read x at
    the pre-rotation position and store dx there); else BatchNorm2d."""
    from shiftgcn import ops
    torch.manual_seed(1)
    B, C, T, V = 6, 16, 20, 25
    xu = torch.randn(B, C, T, V, device=DEV) * 2 + 0.7    # as stored (pre-rotation)
    x = _rot(xu) if per_joint else xu                    # the BatchNorm's logical input
    r = torch.randn(B, C, T, V, device=DEV)
    F = C * V if per_joint else C
    bn = torch.nn.BatchNorm1d(F).to(DEV) if per_joint else torch.nn.BatchNorm2d(C).to(DEV)
    bnr = torch.nn.BatchNorm2d(C).to(DEV)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5); bn.bias.uniform_(-0.5, 0.5)
        bnr.weight.uniform_(0.5, 1.5); bnr.bias.uniform_(-0.5, 0.5)
    bn_ref = type(bn)(F).to(DEV); bn_ref.load_state_dict(bn.state_dict())
    bnr_ref = torch.nn.BatchNorm2d(C).to(DEV); bnr_ref.load_state_dict(bnr.state_dict())
    perm = V if per_joint else 0
    pj = 3 if per_joint else 0
    part = ops.moments(xu, pj)
    st = ops.bn_finalize(part, B, F, T if per_joint else T * V, bn, perm_V=perm)
    rst = ops.bn_finalize(ops.moments(r, False), B, C, T * V, bnr)
    y = ops.bn_apply(xu, st, pj, r=r, rst=rst, relu=True)

    def ref_bn(mod, t, pj):
        if pj:  # BatchNorm1d over (b,t) of features (v, c) -> reference feature v*C + c
            z = t.permute(0, 2, 3, 1).reshape(B * T, V * C)
            return mod(z).view(B, T, V, C).permute(0, 3, 1, 2)
        return mod(t)

    xr = x.clone().requires_grad_(True)
    rr = r.clone().requires_grad_(True)
    yr = torch.relu(ref_bn(bn_ref, xr, per_joint) + ref_bn(bnr_ref, rr, False))
    torch.testing.assert_close(y, yr, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(bn.running_mean, bn_ref.running_mean, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(bn.running_var, bn_ref.running_var, rtol=1e-5, atol=1e-6)
    assert int(bn.num_batches_tracked) == int(bn_ref.num_batches_tracked) == 1
    dy = torch.randn_like(y)
    yr.backward(dy)
    p, rp = ops.bn_bwd_reduce(dy, y, True, xu, st, pj, r=r, rst=rst)
    coef, dg, db = ops.bn_bwd_finalize(p, B, F, B * (T if per_joint else T * V), st, bn,
                                       perm_V=perm)
    rcoef, rdg, rdb = ops.bn_bwd_finalize(rp, B, C, B * T * V, rst, bnr)
    dr = torch.empty_like(r)
    dx = ops.bn_bwd_apply(dy, y, True, xu, coef, pj, r=r, rcoef=rcoef, dr=dr)
    torch.testing.assert_close(_rot(dx) if per_joint else dx, xr.grad, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(dr, rr.grad, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(dg, bn_ref.weight.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(db, bn_ref.bias.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(rdg, bnr_ref.weight.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(rdb, bnr_ref.bias.grad, rtol=1e-4, atol=1e-4)
