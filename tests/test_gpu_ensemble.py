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


def test_ensemble_graph_recaptures_after_weight_change():
    """EnsembleGraph holds no eval-constant launches (they are cached per weight version
    outside the graph): after an in-place weight or running-statistics change, run()
    captures again and still matches the eager forward."""
    e = _our_ensemble()
    from shiftgcn.ensemble import EnsembleGraph
    x = formula.tensor((4, 3, 32, 33, 1), 903, 1.0).to(DEV)
    g = EnsembleGraph(e, x.shape, DEV)
    s0, _ = g.run(x)
    s0 = s0.clone()
    assert g.captures == 1
    with torch.no_grad():
        e.models[2].l3.gcn1.bn.running_var.mul_(2.0)
        e.models[1].l5.tcn1.temporal_linear.weight.mul_(-1.0)
        e.models[0].data_bn.running_mean.add_(0.5)
    s1, l1 = g.run(x)
    se, le = e(x)
    torch.cuda.synchronize()
    assert g.captures == 2
    assert torch.equal(s1, se) and torch.equal(l1, le)
    assert not torch.equal(s0, s1)


# inference recipes (shiftgcn.fused knob EVAL_FOLD)
RECIPES = {"pre-staged": 0, "pre-staged+fold": 1}


@pytest.mark.parametrize("recipe", list(RECIPES))
@pytest.mark.parametrize("cin,cout,stride,residual,V", [(3, 64, 1, False, 25),
                                                        (64, 64, 1, True, 33),
                                                        (64, 128, 2, True, 25),
                                                        (128, 256, 2, True, 33)])
def test_inference_fusions_match_eval_recipe(cin, cout, stride, residual, V, recipe,
                                             monkeypatch):
    """The no-backward recipe (the Shift_gcn tail staged into shift_in, the unit tail in the
    shift_out store and the next-unit gather; optionally the down / residual BatchNorms
    folded into their convs) equals the eval recipe a backward would use."""
    import shiftgcn
    from shiftgcn import fused
    monkeypatch.setattr(fused, "EVAL_FOLD", RECIPES[recipe])
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


def test_eval_constants_track_parameter_and_statistics_updates(monkeypatch):
    """The eval fold of down.1 into down.0 (and residual.bn into residual.conv), the eval
    BatchNorm coefficients and the masks are cached per tensor version: in-place changes of
    the running statistics, of a conv weight or of a Feature_Mask (optimizer steps,
    load_state_dict) are seen by the next inference call."""
    import shiftgcn
    from shiftgcn import fused
    u = shiftgcn.TCN_GCN_unit(64, 128, None, stride=2, residual=True, num_point=25)
    formula.fill_state(u, seed=77)
    u = u.to(DEV).eval()
    x = formula.tensor((2, 64, 16, 25), 78, 1.0).to(DEV)

    def check():
        with torch.no_grad():
            fast = u(x)
        # the eval recipe on a fresh copy of the current state: no cached constants
        v = shiftgcn.TCN_GCN_unit(64, 128, None, stride=2, residual=True, num_point=25)
        v.load_state_dict(u.state_dict())
        v = v.to(DEV).eval()
        ref = v(x.clone().requires_grad_(True)).detach()
        err = (fast - ref).abs().max().item()
        assert err <= 2e-6 * max(1.0, ref.abs().max().item()), err
        return fast

    monkeypatch.setattr(fused, "EVAL_FOLD", 1)
    y0 = check()
    assert "_sgcn_eval_coef" in u.tcn1.bn2.__dict__      # cached
    with torch.no_grad():
        u.gcn1.down[1].running_var.mul_(3.0)
        u.residual.bn.running_mean.add_(0.25)
    y1 = check()
    assert not torch.equal(y0, y1)
    with torch.no_grad():
        u.gcn1.down[0].weight.mul_(-0.5)
    y2 = check()
    with torch.no_grad():
        u.tcn1.bn2.weight.mul_(0.5)
        u.gcn1.bn.running_mean.add_(0.1)
    y3 = check()
    with torch.no_grad():
        u.gcn1.Feature_Mask.add_(0.3)
    y4 = check()
    for a, b in ((y1, y2), (y2, y3), (y3, y4)):
        assert not torch.equal(a, b)


def test_eval_constants_follow_native_training_steps():
    """the training step writes weights (FusedSGD's one launch) and
    running statistics (sgcn_bn_finalize) through raw pointers; those writers advance the
    tensors' version counters, so train epoch -> eval -> train epoch -> eval recomputes
    every cached eval constant (fold, BatchNorm coefficients, masks)."""
    import shiftgcn
    from shiftgcn import train
    torch.manual_seed(5)
    m = shiftgcn.Model(num_class=10, num_point=25, num_person=2, graph="graph.ntu_rgb_d.Graph")
    formula.fill_state(m, seed=9)
    m = m.to(DEV)
    opt = train.build_optimizer(m, base_lr=0.1)
    assert isinstance(opt, train.FusedSGD)
    x = formula.tensor((4, 3, 16, 25, 2), 10, 1.0).to(DEV)
    lab = torch.arange(4, device=DEV) % 10

    def evaluate():
        m.eval()
        with torch.no_grad():
            fast = m(x)
        m.train()
        # a fresh copy of the current state (no cached constants), same eval path
        f = shiftgcn.Model(num_class=10, num_point=25, num_person=2,
                           graph="graph.ntu_rgb_d.Graph")
        f.load_state_dict(m.state_dict())
        f = f.to(DEV).eval()
        with torch.no_grad():
            ref = f(x)
        err = (fast - ref).abs().max().item()
        assert err <= 1e-5 * max(1.0, ref.abs().max().item()), err
        return fast

    outs = []
    for _ in range(3):
        for _ in range(2):
            train.train_step(m, opt, x, lab)
        outs.append(evaluate())
    assert not torch.equal(outs[0], outs[1]) and not torch.equal(outs[1], outs[2])
