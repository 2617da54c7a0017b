"""Shift_gcn.bn's backward partials made by the Shift_tcn.shift_in backward launch
(sgcn_tshift_bwd_gbn + sgcn_bn_bwd_finalize_gbn; reference model/shift_gcn.py:137-141 then
:66-68, shift_cuda_kernel.cu:78-150 for the shift backward):

* the input gradient is bit-identical to sgcn_tshift_bwd's, its plane sums (position
  gradients, Shift_tcn.bn partials) equal up to summation order;
* the per-joint BatchNorm's coefficients and dgamma/dbeta match the two-pass form
  (sgcn_bn_bwd_reduce with the on-the-fly input gradient + sgcn_bn_bwd_finalize) and an
  fp64 torch evaluation of the same sums, within 1e-5 relative;
* unit parity vs the oracle with the fusion off (the default-on path is covered by
  test_gpu_blocks / test_gpu_fullsize).
"""
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu
DEV = "cuda"

# the last two: planes of 8,100 / 7,920 floats need > 32 elements per thread on 256
# threads, so the launcher takes 512 (these raised EINVAL before)
CASES = [(4, 64, 30, 25), (2, 128, 17, 25), (3, 32, 9, 33), (2, 16, 300, 25),
         (2, 16, 324, 25), (2, 16, 240, 33),
         # shifts past the kernel's zero padding (|floor(y)| >= 4, |x| >= 1): the
         # range-checked loop of tshift_bwd_ra_kernel
         (2, 16, 40, 25, "wide")]


def _setup(B, C, T, V, seed, wide=False):
    from shiftgcn import ops
    g = torch.Generator().manual_seed(seed)
    Z = (torch.randn(B, C, T, V, generator=g) * 2 + 0.5).to(DEV)
    H = torch.relu(torch.randn(B, C, T, V, generator=g) + 0.3).to(DEV)
    dAs = torch.randn(B, C, T, V, generator=g).to(DEV)
    xpos = ((torch.rand(C, generator=g) - 0.5) * 2e-8).to(DEV)
    ypos = ((torch.rand(C, generator=g) - 0.5) * (24 if wide else 4)).to(DEV)
    if wide:
        xpos[:4] = torch.tensor([1.5, -2.25, 0.75, -0.5])
    bn_t, bn_g = nn.BatchNorm2d(C).to(DEV), nn.BatchNorm1d(C * V).to(DEV)
    with torch.no_grad():
        bn_t.weight.copy_(torch.rand(C, generator=g) + 0.5)
        bn_t.bias.copy_(torch.randn(C, generator=g))
        bn_g.weight.copy_(torch.rand(C * V, generator=g) + 0.5)
        bn_g.bias.copy_(torch.randn(C * V, generator=g))
    ast = ops.bn_finalize(ops.moments(H, False), B, C, T * V, bn_t)
    # Z is the gcn contraction output before its shift_out (per_joint = 3 layout)
    zst = ops.bn_finalize(ops.moments(Z, 3), B, C * V, T, bn_g, perm_V=V)
    return Z, H, dAs, xpos, ypos, bn_t, bn_g, ast, zst


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max()) / (float(b.abs().max()) + 1e-30)


@pytest.mark.parametrize("case", CASES, ids=["x".join(map(str, c)) for c in CASES])
def test_gbn_matches_two_pass(case):
    from shiftgcn import ops
    B, C, T, V = case[:4]
    Z, H, dAs, xpos, ypos, bn_t, bn_g, ast, zst = _setup(B, C, T, V, sum(case[:4]),
                                                         wide=len(case) > 4)
    dA1, gx1, gy1, part1 = ops.tshift_bwd(dAs, H, xpos, ypos, 1, scale=ast.scale,
                                          shift=ast.shift, bn_stats=ast)
    dA2, gx2, gy2, part2, z6 = ops.tshift_bwd_gbn(dAs, H, xpos, ypos, ast, Z, zst)
    torch.cuda.synchronize()
    # the input gradient is bit-identical; the plane sums (position gradients, Shift_tcn.bn
    # partials) are the same sums over a joint-aligned thread assignment, so only their
    # summation order differs (the position gradients keep only the sign of theirs)
    assert torch.equal(dA1, dA2)
    assert int((gx1 != gx2).sum() + (gy1 != gy2).sum()) <= 1
    assert _rel(part2, part1) < 1e-6
    coefA, _, _ = ops.bn_bwd_finalize(part1, B, C, B * T * V, ast, bn_t)
    # two-pass reference: reduce over (dA, H, Z) with the on-the-fly input gradient
    rp, _ = ops.bn_bwd_reduce(dA1, H, True, Z, zst, 3, dy_coef=coefA)
    c_ref, dg_ref, db_ref = ops.bn_bwd_finalize(rp, B, C * V, B * T, zst, bn_g, perm_V=V)
    c_new, dg_new, db_new = ops.bn_bwd_finalize_gbn(z6, B, C, V, B * T, coefA, ast, zst, bn_g)
    # fp64 evaluation of the same sums (reference feature order v*C + c)
    k = coefA.double()
    gd = (k[0].view(1, C, 1, 1) * dA1.double() + k[1].view(1, C, 1, 1) * H.double()
          + k[2].view(1, C, 1, 1)) * (H > 0)
    idx = (torch.arange(V, device=DEV)[None, :] - torch.arange(C, device=DEV)[:, None]) % V
    Zl = Z.gather(3, idx.view(1, C, 1, V).expand(B, C, T, V))      # logical (rotated) Z
    zh = (Zl.double() - zst.mean.double().view(1, C, 1, V)) * zst.invstd.double().view(1, C, 1, V)
    sg = gd.sum((0, 2)).t().reshape(-1)                 # (C, V) -> (V, C) -> v*C + c
    sgx = (gd * zh).sum((0, 2)).t().reshape(-1)
    torch.cuda.synchronize()
    assert _rel(db_new, sg) < 1e-5 and _rel(dg_new, sgx) < 1e-5
    assert _rel(db_new, db_ref) < 1e-5 and _rel(dg_new, dg_ref) < 1e-5
    assert _rel(c_new[0], c_ref[0]) == 0.0                # k1 = gamma * invstd, same floats
    assert _rel(c_new[1], c_ref[1]) < 1e-5 and _rel(c_new[2], c_ref[2]) < 1e-5


def test_unit_parity_with_gbn_off(monkeypatch):
    import formula
    import shiftgcn
    from oracle import model_oracle as mo
    from shiftgcn import fused
    from test_gpu_blocks import _compare
    monkeypatch.setattr(fused, "GBN_FUSION", 0)
    ref = mo.TCN_GCN_unit(64, 64, None, stride=1, num_point=25)
    formula.fill_state(ref, seed=23)
    ours = shiftgcn.TCN_GCN_unit(64, 64, None, stride=1, num_point=25).to(DEV)
    ours.load_state_dict(ref.state_dict())
    x = formula.tensor((3, 64, 14, 25), 71, 1.0)
    g = formula.tensor((3, 64, 14, 25), 72, 1.0)
    xr = x.clone().requires_grad_(True)
    yr = ref(xr)
    yr.backward(g)
    xo = x.to(DEV).requires_grad_(True)
    yo = ours(xo)
    yo.backward(g.to(DEV))
    torch.cuda.synchronize()
    _compare(ref, ours, xr, yr, xo, yo, "gbn-off")


def test_gbn_path_taken_in_model(monkeypatch):
    """Every unit takes the fused path (l1 / l5 / l8 with their down BatchNorm's sums too):
    no bn_bwd_reduce on a per-joint BatchNorm remains (only the unit-tail reduces)."""
    import shiftgcn
    from shiftgcn import ops
    calls = {"gbn": 0, "pj_reduce": 0}
    real_gbn, real_red = ops.tshift_bwd_gbn, ops.bn_bwd_reduce

    def spy_gbn(*a, **k):
        calls["gbn"] += 1
        return real_gbn(*a, **k)

    def spy_red(dy, y, relu, x, st, per_joint, *a, **k):
        calls["pj_reduce"] += int(bool(per_joint))
        return real_red(dy, y, relu, x, st, per_joint, *a, **k)

    monkeypatch.setattr(ops, "tshift_bwd_gbn", spy_gbn)
    monkeypatch.setattr(ops, "bn_bwd_reduce", spy_red)
    m = shiftgcn.Model(num_class=60, num_point=25, num_person=2,
                       graph="graph.ntu_rgb_d.Graph").to(DEV).train()
    m(torch.randn(2, 3, 16, 25, 2, device=DEV)).sum().backward()
    torch.cuda.synchronize()
    assert calls == {"gbn": 10, "pj_reduce": 0}, calls


@pytest.mark.parametrize("case", [(4, 64, 30, 25), (2, 16, 300, 25), (3, 32, 9, 33),
                                  (2, 16, 40, 25, "wide")],
                         ids=["4x64x30x25", "2x16x300x25", "3x32x9x33", "wide"])
def test_gbn_down_sums_match_two_pass(case):
    """With a down conv (H = relu(bn(Z) + bnd(D))), the down BatchNorm's backward sums from
    the same launch (sgcn_tshift_bwd_gbn d_part, finalized with V = 1) match the two-pass
    form (sgcn_bn_bwd_reduce with the residual BatchNorm + sgcn_bn_bwd_finalize) and fp64;
    the gcn BatchNorm's sums are unchanged by the extra operand."""
    from shiftgcn import ops
    B, C, T, V = case[:4]
    Z, H, dAs, xpos, ypos, bn_t, bn_g, ast, zst = _setup(B, C, T, V, 3 + sum(case[:4]),
                                                         wide=len(case) > 4)
    g = torch.Generator().manual_seed(11)
    D = (torch.randn(B, C, T, V, generator=g) * 1.5 - 0.2).to(DEV)
    bn_d = nn.BatchNorm2d(C).to(DEV)
    with torch.no_grad():
        bn_d.weight.copy_(torch.rand(C, generator=g) + 0.5)
        bn_d.bias.copy_(torch.randn(C, generator=g))
    dst = ops.bn_finalize(ops.moments(D, False), B, C, T * V, bn_d)
    dA1, gx1, gy1, part1, z6 = ops.tshift_bwd_gbn(dAs, H, xpos, ypos, ast, Z, zst)
    dA2, gx2, gy2, part2, z6d, d6 = ops.tshift_bwd_gbn(dAs, H, xpos, ypos, ast, Z, zst,
                                                        down=(D, dst))
    torch.cuda.synchronize()
    assert torch.equal(dA1, dA2)
    if -(-T * V // ((256 // V) * V)) <= 24:   # the same 256-thread launch for both forms
        assert torch.equal(part1, part2) and torch.equal(z6, z6d)
    else:
        # planes that need 32 elements per thread on 256 threads run the GBD form on 512
        # threads x 16 (register pressure, tshift.hip SGCN_GBD_SPLIT): the same plane sums,
        # added in another order
        assert _rel(part2, part1) < 1e-6 and _rel(z6d, z6) < 1e-6
    coefA, _, _ = ops.bn_bwd_finalize(part1, B, C, B * T * V, ast, bn_t)
    rp, rpart = ops.bn_bwd_reduce(dA1, H, True, Z, zst, 3, r=D, rst=dst, dy_coef=coefA)
    c_ref, dg_ref, db_ref = ops.bn_bwd_finalize(rpart, B, C, B * T * V, dst, bn_d)
    c_new, dg_new, db_new = ops.bn_bwd_finalize_gbn(d6, B, C, 1, B * T * V, coefA, ast, dst,
                                                    bn_d)
    k = coefA.double()
    gd = (k[0].view(1, C, 1, 1) * dA1.double() + k[1].view(1, C, 1, 1) * H.double()
          + k[2].view(1, C, 1, 1)) * (H > 0)
    dh = (D.double() - dst.mean.double().view(1, C, 1, 1)) * dst.invstd.double().view(1, C, 1, 1)
    torch.cuda.synchronize()
    assert _rel(db_new, gd.sum((0, 2, 3))) < 1e-5
    assert _rel(dg_new, (gd * dh).sum((0, 2, 3))) < 1e-5
    assert _rel(db_new, db_ref) < 1e-5 and _rel(dg_new, dg_ref) < 1e-5
    assert _rel(c_new[0], c_ref[0]) == 0.0
    assert _rel(c_new[1], c_ref[1]) < 1e-5 and _rel(c_new[2], c_ref[2]) < 1e-5


# planes the LDS-staged stride-1 backward does not take (W > 64, or more than 16,384
# floats): sgcn_tshift_bwd falls back to the global-tap kernel, whose BatchNorm partials
# must read the statistics of the plane's OWN channel (a bug there read them at
# blockIdx % C, and no test reached this kernel with bn_stats)
@pytest.mark.parametrize("shape", [(2, 6, 12, 70), (1, 3, 700, 25)],
                         ids=["W70", "HW17500"])
def test_global_tap_backward_bn_partials(shape):
    from shiftgcn import ops
    B, C, T, V = shape
    g = torch.Generator().manual_seed(B * 1000 + C * 100 + T + V)
    H = (torch.randn(B, C, T, V, generator=g) * 1.5 + 0.25).to(DEV)
    dAs = torch.randn(B, C, T, V, generator=g).to(DEV)
    xpos = ((torch.rand(C, generator=g) - 0.5) * 2e-8).to(DEV)
    ypos = ((torch.rand(C, generator=g) - 0.5) * 4).to(DEV)
    bn = nn.BatchNorm2d(C).to(DEV)
    with torch.no_grad():
        bn.weight.copy_(torch.rand(C, generator=g) + 0.5)
        bn.bias.copy_(torch.randn(C, generator=g))
    st = ops.bn_finalize(ops.moments(H, False), B, C, T * V, bn)
    # distinct per-channel statistics, so reading another channel's shows
    assert float(st.mean.std()) > 0
    gin, gx, gy, part = ops.tshift_bwd(dAs, H, xpos, ypos, 1, scale=st.scale, shift=st.shift,
                                       bn_stats=st)
    torch.cuda.synchronize()
    gd = gin.double()
    xhat = (H.double() - st.mean.double().view(1, C, 1, 1)) * st.invstd.double().view(1, C, 1, 1)
    ref = torch.stack([gd.sum((2, 3)), (gd * xhat).sum((2, 3))], -1).reshape(-1)
    assert _rel(part, ref) < 1e-5
    # the input gradient itself (independent of the affine taps): bit-exact vs the oracle
    from oracle import shift_oracle as so
    exp = so.shift_bottom_backward(dAs.cpu().numpy(), xpos.cpu().numpy(), ypos.cpu().numpy(),
                                   T, 1)
    assert torch.equal(gin.cpu(), torch.from_numpy(exp))
