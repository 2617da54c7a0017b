"""Training BatchNorm finalizes folded into their consumers (round 4, sgcn_bn_fold): the
consumer's plane workgroups merge the batch partials in sgcn_bn_finalize's order, so every
result must be BIT-identical to the separate finalize launch — the coefficients, the
consumer's output, the running statistics and num_batches_tracked — including the shapes
whose consumer falls back to the separate launch (W > 64, model.shift_gcn.py:55-57, 85, 38
BatchNorms; reference semantics are those of nn.BatchNorm2d in train())."""
import copy

import pytest
import torch

import formula

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _bn(C, seed):
    g = torch.Generator().manual_seed(seed)
    bn = torch.nn.BatchNorm2d(C).to(DEV)
    with torch.no_grad():
        bn.weight.copy_(torch.rand(C, generator=g) + 0.5)
        bn.bias.copy_(torch.randn(C, generator=g))
        bn.running_mean.copy_(torch.randn(C, generator=g))
        bn.running_var.copy_(torch.rand(C, generator=g) + 0.5)
    return bn


@pytest.mark.parametrize("B,C,T,V", [(4, 16, 30, 25), (3, 8, 12, 70), (2, 64, 300, 25),
                                     (3, 32, 75, 33)])
def test_shift_with_folded_finalize(B, C, T, V, monkeypatch):
    from shiftgcn import ops
    g = torch.Generator().manual_seed(B + C + T + V)
    H = (torch.randn(B, C, T, V, generator=g) + 0.3).to(DEV)
    xpos = ((torch.rand(C, generator=g) - 0.5) * 2e-8).to(DEV)
    ypos = ((torch.rand(C, generator=g) - 0.5) * 4).to(DEV)
    part = ops.moments(H, False)
    res = []
    for fold in (0, 1):
        monkeypatch.setattr(ops, "FOLD_FINALIZE", fold)
        bn = _bn(C, 5)
        st = ops.bn_finalize(part, B, C, T * V, bn, defer=True)
        assert st.pending == bool(fold)
        out = ops.tshift_fwd(H, xpos, ypos, 1, affine=st)
        torch.cuda.synchronize()
        res.append((out, st.mean.clone(), st.invstd.clone(), st.scale.clone(),
                    st.shift.clone(), bn.running_mean.clone(), bn.running_var.clone(),
                    int(bn.num_batches_tracked)))
    for a, b in zip(res[0][:-1], res[1][:-1]):
        assert torch.equal(a, b)
    assert res[0][-1] == res[1][-1] == 1


@pytest.mark.parametrize("B,C,T,V", [(4, 16, 30, 25), (3, 8, 12, 70), (2, 64, 150, 25)])
@pytest.mark.parametrize("which", ["main", "residual", "both"])
def test_apply_with_folded_finalizes(B, C, T, V, which, monkeypatch):
    from shiftgcn import ops
    g = torch.Generator().manual_seed(7 * B + C + T + V)
    S = torch.randn(B, C, T, V, generator=g).to(DEV)
    R = (torch.randn(B, C, T, V, generator=g) * 2).to(DEV)
    ps, pr = ops.moments(S, False), ops.moments(R, False)
    res = []
    for fold in (0, 1):
        monkeypatch.setattr(ops, "FOLD_FINALIZE", fold)
        bn1, bn2 = _bn(C, 11), _bn(C, 12)
        st = ops.bn_finalize(ps, B, C, T * V, bn1, defer=which in ("main", "both"))
        rst = ops.bn_finalize(pr, B, C, T * V, bn2, defer=which in ("residual", "both"))
        y, ys = ops.bn_apply(S, st, False, r=R, rst=rst, relu=True, out_stats=True)
        torch.cuda.synchronize()
        res.append([y, ys] + [t.clone() for t in (st.mean, st.invstd, st.scale, st.shift,
                                                  rst.mean, rst.invstd, rst.scale, rst.shift,
                                                  bn1.running_mean, bn1.running_var,
                                                  bn2.running_mean, bn2.running_var,
                                                  bn1.num_batches_tracked,
                                                  bn2.num_batches_tracked)])
    for a, b in zip(res[0], res[1]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("cfg", ["ntu", "mp"])
def test_training_steps_bit_identical_with_folded_finalizes(cfg, monkeypatch):
    """Two SGD steps of the whole model with the per-channel finalizes folded and not:
    bit-identical logits, gradients, parameters and BatchNorm buffers."""
    import shiftgcn
    from shiftgcn import ops, train
    V, M, nc, graph = ((25, 2, 60, "graph.ntu_rgb_d.Graph") if cfg == "ntu" else
                       (33, 1, 2, "graph.mediapipe_pose.Graph"))
    m0 = shiftgcn.Model(num_class=nc, num_point=V, num_person=M, graph=graph)
    formula.fill_state(m0, seed=91)
    x = formula.tensor((4, 3, 32, V, M), 92, 1.0).to(DEV)
    y = (torch.arange(4) * 5 % nc).to(DEV)
    out = []
    for fold in (0, 1):
        monkeypatch.setattr(ops, "FOLD_FINALIZE", fold)
        m = copy.deepcopy(m0).to(DEV).train()
        opt = train.build_optimizer(m, base_lr=0.1)
        logits = []
        for _ in range(2):
            logits.append(m(x).detach())
            loss = torch.nn.functional.cross_entropy(m(x), y)
            opt.zero_grad(set_to_none=True)
            loss.backward()
            opt.step()
        torch.cuda.synchronize()
        out.append((logits, {k: v.detach().clone() for k, v in m.state_dict().items()},
                    {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}))
    (l0, s0, g0), (l1, s1, g1) = out
    for a, b in zip(l0, l1):
        assert torch.equal(a, b)
    assert s0.keys() == s1.keys() and g0.keys() == g1.keys()
    for k in s0:
        assert torch.equal(s0[k], s1[k]), k
    for k in g0:
        assert torch.equal(g0[k], g1[k]), k


@pytest.mark.parametrize("B,C,T,V", [(4, 16, 30, 25), (3, 8, 12, 70), (2, 64, 150, 25)])
def test_backward_apply_with_folded_finalizes(B, C, T, V, monkeypatch):
    """bn2 + residual BatchNorm backward finalizes folded into the unit tail's backward apply
    (sgcn_bn_bwd_apply_fold): bit-identical coefficients, dgamma/dbeta, dx and dr."""
    from shiftgcn import ops
    g = torch.Generator().manual_seed(3 * B + C + T + V)
    S = torch.randn(B, C, T, V, generator=g).to(DEV)
    R = (torch.randn(B, C, T, V, generator=g) * 2).to(DEV)
    dy = torch.randn(B, C, T, V, generator=g).to(DEV)
    bn1, bn2 = _bn(C, 21), _bn(C, 22)
    st = ops.bn_finalize(ops.moments(S, False), B, C, T * V, bn1)
    rst = ops.bn_finalize(ops.moments(R, False), B, C, T * V, bn2)
    y = ops.bn_apply(S, st, False, r=R, rst=rst, relu=True)
    part, rpart = ops.bn_bwd_reduce(dy, y, True, S, st, False, r=R, rst=rst)
    res = []
    for fold in (0, 1):
        monkeypatch.setattr(ops, "FOLD_FINALIZE", fold)
        coef, dg, db = ops.bn_bwd_finalize(part, B, C, B * T * V, st, bn1, defer=True)
        rcoef, rdg, rdb = ops.bn_bwd_finalize(rpart, B, C, B * T * V, rst, bn2, defer=True)
        assert isinstance(coef, ops.PendingCoef) == bool(fold)
        dx, dr = torch.empty_like(S), torch.empty_like(R)
        ops.bn_bwd_apply(dy, y, True, S, coef, False, r=R, rcoef=rcoef, dr=dr, dx=dx)
        torch.cuda.synchronize()
        ct = coef.t if fold else coef
        rt = rcoef.t if fold else rcoef
        res.append([dx, dr, ct.clone(), rt.clone(), dg.clone(), db.clone(), rdg.clone(),
                    rdb.clone()])
    for a, b in zip(res[0], res[1]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("B,C,T,V", [(4, 16, 30, 25), (2, 64, 300, 25), (3, 32, 75, 33)])
def test_shift_out_backward_with_folded_finalize(B, C, T, V, monkeypatch):
    """bn2's backward finalize folded into the shift_out backward (sgcn_tshift_bwd_bnin_fold,
    shift_gcn.py:72-73 + 161-162): bit-identical input and position gradients, coefficients
    and dgamma/dbeta."""
    from shiftgcn import ops
    g = torch.Generator().manual_seed(5 * B + C + T + V)
    R = torch.relu(torch.randn(B, C, T, V, generator=g) + 0.2).to(DEV)
    xpos = ((torch.rand(C, generator=g) - 0.5) * 2e-8).to(DEV)
    ypos = ((torch.rand(C, generator=g) - 0.5) * 4).to(DEV)
    bn = _bn(C, 31)
    stats = torch.empty(B * C * 2, device=DEV)
    S = ops.tshift_fwd(R, xpos, ypos, 1, stats=stats)
    sst = ops.bn_finalize(stats, B, C, T * V, bn)
    out = ops.bn_apply(S, sst, False, relu=True)
    dout = torch.randn(B, C, T, V, generator=g).to(DEV)
    part, _ = ops.bn_bwd_reduce(dout, out, True, S, sst, False)
    res = []
    for fold in (0, 1):
        monkeypatch.setattr(ops, "FOLD_FINALIZE", fold)
        coef, dg, db = ops.bn_bwd_finalize(part, B, C, B * T * V, sst, bn, defer=True)
        gin, gx, gy = ops.tshift_bwd_bnin(dout, out, S, coef, R, xpos, ypos)
        torch.cuda.synchronize()
        ct = coef.t if fold else coef
        res.append([gin, gx, gy, ct.clone(), dg.clone(), db.clone()])
    for a, b in zip(res[0], res[1]):
        assert torch.equal(a, b)
