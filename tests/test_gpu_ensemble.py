"""GPU parity of the ensemble path (BASELINE config 4): the fused modality/head kernel
(bit-exact streams; data_bn within fp32 rounding) and the batched 4-model ensemble, eager
and hipGraph-replayed, against the oracle and the reference's own fused scores
(tests/golden/ensemble_fixtures.npz)."""
import numpy as np
import pytest
import torch

import formula
from oracle import ensemble_oracle as eo
from test_oracle_ensemble import STREAMS, oracle_models

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("N,T,V,M", [(5, 37, 33, 1), (3, 20, 25, 2), (1, 1, 33, 1),
                                     (0, 8, 33, 1)])
def test_modalities_bit_exact(N, T, V, M):
    from shiftgcn import ensemble as ens
    pairs = ens.MEDIAPIPE_BONE_PAIRS if V == 33 else ens.NTU_BONE_PAIRS
    joint = formula.tensor((N, 3, T, V, M), 11 + N + V, 1.0)
    parent = torch.from_numpy(ens.parent_table(pairs, V)).to(DEV)
    ref = eo.derive_modalities(joint.numpy(), pairs)
    got = ens.derive_modalities(joint.to(DEV), parent, planes=False)
    gotp = ens.derive_modalities(joint.to(DEV), parent, planes=True)
    for s, g, gp in zip(STREAMS, got, gotp):
        assert np.array_equal(g.cpu().numpy(), ref[s]), s
        planes = ref[s].transpose(0, 4, 1, 2, 3).reshape(N * M, 3, T, V)
        assert np.array_equal(gp.cpu().numpy(), planes), s


def test_modalities_with_data_bn_head():
    """planes + data_bn == the Model.forward head (permute, BatchNorm1d eval, permute)."""
    import shiftgcn
    from shiftgcn import ensemble as ens
    N, T, V, M = 4, 16, 25, 2
    models = []
    for k in range(4):
        m = shiftgcn.Model(num_class=60, num_point=V, num_person=M,
                           graph="graph.ntu_rgb_d.Graph")
        formula.fill_state(m, seed=31 + k)
        models.append(m.to(DEV).eval())
    e = ens.Ensemble(models, bone_pairs=ens.NTU_BONE_PAIRS).to(DEV)
    joint = formula.tensor((N, 3, T, V, M), 77, 1.0).to(DEV)
    streams = ens.derive_modalities(joint, e.parent, planes=True, data_bn=e._data_bn_coef())
    raw = ens.derive_modalities(joint, e.parent, planes=False)
    for m, xs, xr in zip(models, streams, raw):
        with torch.no_grad():
            x = xr.permute(0, 4, 3, 1, 2).contiguous().view(N, M * V * 3, T)
            x = m.data_bn(x).view(N, M, V, 3, T).permute(0, 1, 3, 4, 2).reshape(N * M, 3, T, V)
        err = (xs - x).abs().max().item()
        assert err <= 2e-6 * max(1.0, x.abs().max().item()), err


def _our_ensemble():
    import shiftgcn
    from shiftgcn import ensemble as ens
    models = []
    for k in range(4):
        m = shiftgcn.Model(num_class=2, num_point=33, num_person=1,
                           graph="graph.mediapipe_pose.Graph")
        formula.fill_state(m, seed=701 + 13 * k)
        models.append(m.to(DEV).eval())
    return ens.Ensemble(models).to(DEV)


def test_ensemble_matches_reference_scores(golden):
    fx = golden("ensemble_fixtures.npz")
    e = _our_ensemble()
    wins = torch.from_numpy(fx["ens_windows"]).to(DEV)        # (W, 3, T, 33, 1)
    scores, fused = e(wins)
    assert np.abs(scores.cpu().numpy() - fx["ens_scores"]).max() < 1e-5
    ref_fused = sum(np.float32(a) * fx[f"ens_logits_{s}"] for a, s in
                    zip(fx["weights"], STREAMS))
    assert np.abs(fused.cpu().numpy() - ref_fused).max() < 1e-4
    # the batch is computed as one: each window alone gives the same scores
    s0, _ = e(wins[1:2])
    assert abs(float(s0[0]) - float(scores[1])) < 1e-6


def test_ensemble_graph_replay_matches_eager():
    e = _our_ensemble()
    N, T = 6, 48
    from shiftgcn.ensemble import EnsembleGraph
    x1 = formula.tensor((N, 3, T, 33, 1), 901, 1.0).to(DEV)
    x2 = formula.tensor((N, 3, T, 33, 1), 902, 1.0).to(DEV)
    ens_graph = EnsembleGraph(e, x1.shape, DEV)
    for x in (x1, x2, x1):
        s_eager, l_eager = e(x)
        s_g, l_g = ens_graph.run(x)
        torch.cuda.synchronize()
        assert torch.equal(s_g, s_eager) and torch.equal(l_g, l_eager)


# inference recipes (shiftgcn.fused knobs): (EVAL_GCN_EPI, EVAL_TSHIFT_FUSION_MIN_C)
# (EVAL_GCN_EPI, EVAL_TSHIFT_FUSION_MIN_C, EVAL_FOLD)
RECIPES = {"pre-staged": (0, 512, 0), "pre-staged+fold": (0, 512, 1),
           "gcn-epilogue": (1, 512, 1), "epilogue+tshift-fused": (1, 0, 1)}


@pytest.mark.parametrize("recipe", list(RECIPES))
@pytest.mark.parametrize("cin,cout,stride,residual,V", [(3, 64, 1, False, 25),
                                                        (64, 64, 1, True, 33),
                                                        (64, 128, 2, True, 25),
                                                        (128, 256, 2, True, 33)])
def test_inference_fusions_match_eval_recipe(cin, cout, stride, residual, V, recipe,
                                             monkeypatch):
    """The no-backward recipes (round 1: Shift_gcn tail staged into shift_in; round 4: that
    tail in the gcn contraction's epilogue with the down / residual BatchNorms folded into
    their convs, optionally shift_in formed inside temporal_linear's staging; always the unit
    tail in the shift_out store and the next-unit gather) equal the eval recipe a backward
    would use."""
    import shiftgcn
    from shiftgcn import fused
    epi, minc, fold = RECIPES[recipe]
    monkeypatch.setattr(fused, "EVAL_GCN_EPI", epi)
    monkeypatch.setattr(fused, "EVAL_TSHIFT_FUSION_MIN_C", minc)
    monkeypatch.setattr(fused, "EVAL_FOLD", fold)
    torch.manual_seed(3)
    u = shiftgcn.TCN_GCN_unit(cin, cout, None, stride=stride, residual=residual,
                              num_point=V)
    formula.fill_state(u, seed=40 + cin + cout)
    u = u.to(DEV).eval()
    x = formula.tensor((3, cin, 20, V), 50 + cout, 1.0).to(DEV)
    with torch.no_grad():
        fused = u(x)
    xr = x.clone().requires_grad_(True)
    ref = u(xr).detach()
    err = (fused - ref).abs().max().item()
    assert err <= 2e-6 * max(1.0, ref.abs().max().item()), err


@pytest.mark.parametrize("epi", [0, 1])
def test_folded_conv_bn_tracks_parameter_and_statistics_updates(epi, monkeypatch):
    """The eval fold of down.1 into down.0 (and residual.bn into residual.conv) is cached
    per tensor version: in-place changes of the running statistics or of the conv weight
    (optimizer steps, load_state_dict) are seen by the next inference call."""
    import shiftgcn
    from shiftgcn import fused
    u = shiftgcn.TCN_GCN_unit(64, 128, None, stride=2, residual=True, num_point=25)
    formula.fill_state(u, seed=77)
    u = u.to(DEV).eval()
    x = formula.tensor((2, 64, 16, 25), 78, 1.0).to(DEV)

    def check():
        with torch.no_grad():
            fast = u(x)
        ref = u(x.clone().requires_grad_(True)).detach()
        err = (fast - ref).abs().max().item()
        assert err <= 2e-6 * max(1.0, ref.abs().max().item()), err
        return fast

    monkeypatch.setattr(fused, "EVAL_GCN_EPI", epi)
    monkeypatch.setattr(fused, "EVAL_FOLD", 1)
    y0 = check()
    with torch.no_grad():
        u.gcn1.down[1].running_var.mul_(3.0)
        u.residual.bn.running_mean.add_(0.25)
    y1 = check()
    assert not torch.equal(y0, y1)
    with torch.no_grad():
        u.gcn1.down[0].weight.mul_(-0.5)
    check()


@pytest.mark.parametrize("M,K,T,V,rsign", [(64, 64, 20, 25, 1), (128, 64, 12, 33, 1),
                                           (256, 128, 9, 25, 1), (64, 3, 7, 25, 0)])
def test_pw_fwd_bn_res_matches_torch(M, K, T, V, rsign):
    """sgcn_pw_fwd_bn_res vs an fp64 torch evaluation: relu((W x + b) * s[m, v'] + t[m, v']
    + res) with v' the stored (shift_out-rotated) joint."""
    from shiftgcn import ops
    g = torch.Generator().manual_seed(M + K + T + V)
    B = 3
    x = torch.randn(B, K, T, V, generator=g)
    w = torch.randn(K, M, generator=g) / K ** 0.5          # Linear_weight (C_in, C_out)
    b = torch.randn(M, generator=g)
    sc = torch.rand(M * V, generator=g) + 0.5
    sh = torch.randn(M * V, generator=g)
    res = torch.randn(B, M, T, V, generator=g)

    class St:
        pass
    st = St()
    st.scale, st.shift = sc.to(DEV), sh.to(DEV)
    y = torch.empty(B, M, T, V, device=DEV)
    ops.pw_fwd_bn_res(w.to(DEV), True, b.to(DEV), ops.PlaneView(x.to(DEV)), st, res.to(DEV),
                      ops.PlaneView(y, 1, rsign), M, K, T, V)
    z = torch.einsum("bktv,km->bmtv", x.double(), w.double()) + b.double().view(1, M, 1, 1)
    # store joint v' = (v + rsign*m) mod V
    vv = (torch.arange(V).view(1, V) + rsign * torch.arange(M).view(M, 1)) % V   # [m, v]
    zr = torch.zeros_like(z)
    zr.scatter_(3, vv.view(1, M, 1, V).expand(B, M, T, V), z)
    ref = torch.relu(zr * sc.double().view(1, M, 1, V) + sh.double().view(1, M, 1, V)
                     + res.double())
    err = (y.cpu().double() - ref).abs().max().item()
    assert err <= 2e-5 * max(1.0, ref.abs().max().item()), err
