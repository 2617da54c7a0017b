"""GPU parity of the fused HIP blocks against the CPU oracle (itself pinned to the
reference modules) and the committed golden fixtures.

Tolerance (fp32, north_star: 1e-5): outputs and input gradients within 2e-5 relative to
the tensor's max magnitude; parameter gradients (long reductions) within 1e-4 relative;
shift-position gradients (sign-normalised, +-0.01) bit-exact except where the reduced
position gradient is within float rounding of zero (<= 1 channel allowed).
"""
import numpy as np
import pytest
import torch

import formula
from gen_fixtures import (BLOCK_CASES, MODEL_CASES, block_case_inputs, build_block,
                          model_case_inputs)
from oracle import model_oracle as mo

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel_close(a, b, tol, what="", floor=2e-5):
    """max|a-b| <= tol*max|b| + floor. The absolute floor covers gradients that are
    mathematically zero (a conv/linear bias feeding straight into a BatchNorm) and are
    pure rounding noise on both sides."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    scale = float(np.abs(b).max()) if b.size else 0.0
    err = float(np.abs(a - b).max()) if a.size else 0.0
    assert err <= tol * scale + floor, f"{what}: max err {err:.3e} vs scale {scale:.3e}"


def zero_by_construction(name):
    """Gradients that are mathematically zero: a bias added right before a BatchNorm over
    the same features (Linear_bias before gcn.bn: shift_gcn.py:132-137; the 1x1 conv bias
    before down.1 / residual.bn). Both sides hold only rounding noise; check they are tiny."""
    return name.endswith(("Linear_bias", "down.0.bias")) or name in ("conv.bias",
                                                                     "residual.conv.bias")


def _shift_grads_close(a, b, what):
    a = np.asarray(a)
    b = np.asarray(b)
    assert (a != b).sum() <= 1, f"{what}: {(a != b).sum()} position-grad mismatches"


def _pair(kind, cin, cout, V, stride, seed):
    import shiftgcn
    ref = build_block(mo, kind, cin, cout, V, stride)
    formula.fill_state(ref, seed=seed)
    ours = build_block(shiftgcn, kind, cin, cout, V, stride).to(DEV)
    ours.load_state_dict(ref.state_dict())
    ref.train()
    ours.train()
    return ref, ours


def _run_pair(ref, ours, x, g):
    xr = x.clone().requires_grad_(True)
    yr = ref(xr)
    yr.backward(g)
    xo = x.to(DEV).requires_grad_(True)
    yo = ours(xo)
    yo.backward(g.to(DEV))
    torch.cuda.synchronize()
    return xr, yr, xo, yo


def _compare(ref, ours, xr, yr, xo, yo, tag, train=True):
    _rel_close(yo.detach().cpu(), yr.detach(), 2e-5, f"{tag} out")
    _rel_close(xo.grad.cpu(), xr.grad, 2e-5, f"{tag} dx")
    po = dict(ours.named_parameters())
    for n, p in ref.named_parameters():
        if p.grad is None:
            assert po[n].grad is None, n
            continue
        go = po[n].grad.cpu()
        if n.endswith(("xpos", "ypos")):
            _shift_grads_close(go.numpy(), p.grad.numpy(), f"{tag} {n}")
        elif train and zero_by_construction(n):   # (running-stats BN keeps bias grads)
            assert float(go.abs().max()) < 1e-3 and float(p.grad.abs().max()) < 1e-3, n
        else:
            _rel_close(go, p.grad, 1e-4, f"{tag} grad {n}")
    bo = dict(ours.named_buffers())
    for n, b in ref.named_buffers():
        if b.dtype.is_floating_point:
            _rel_close(bo[n].cpu(), b, 2e-5, f"{tag} buffer {n}")
        else:
            assert int(bo[n]) == int(b), n


@pytest.mark.parametrize("case", BLOCK_CASES, ids=[c[0] for c in BLOCK_CASES])
def test_block_matches_golden_fixture(golden, case):
    """Same deterministic weights/inputs the reference modules ran on."""
    import shiftgcn
    fx = golden("block_fixtures.npz")
    name, kind, cin, cout, NM, T, V, stride = case
    m = build_block(shiftgcn, kind, cin, cout, V, stride)
    formula.fill_state(m, seed=31 + sum(map(ord, name)))
    m = m.to(DEV).train()
    x, g = block_case_inputs(*case)
    xo = x.to(DEV).requires_grad_(True)
    y = m(xo)
    y.backward(g.to(DEV))
    _rel_close(y.detach().cpu(), fx[f"blk_{name}_out"], 2e-5, "out")
    _rel_close(xo.grad.cpu(), fx[f"blk_{name}_gx"], 2e-5, "dx")
    for pn, p in m.named_parameters():
        key = f"blk_{name}_grad.{pn}"
        if p.grad is None:
            continue
        if pn.endswith(("xpos", "ypos")):
            _shift_grads_close(p.grad.cpu().numpy(), fx[key], pn)
        elif zero_by_construction(pn):
            assert float(p.grad.abs().max()) < 1e-3 and float(np.abs(fx[key]).max()) < 1e-3
        else:
            _rel_close(p.grad.cpu(), fx[key], 1e-4, pn)
    for bn, b in m.named_buffers():
        if b.dtype.is_floating_point:
            _rel_close(b.cpu(), fx[f"blk_{name}_buf.{bn}"], 2e-5, bn)


REAL_CASES = [
    # (kind, cin, cout, NM, T, V, stride) at the model's real channel widths
    ("gcn", 3, 64, 4, 20, 25, 1),
    ("gcn", 64, 64, 4, 20, 25, 1),
    ("gcn", 64, 128, 3, 12, 25, 1),
    ("gcn", 128, 256, 2, 10, 33, 1),
    ("tcn", 64, 64, 4, 20, 25, 1),
    ("tcn", 128, 128, 3, 16, 25, 2),
    ("unit", 64, 128, 3, 20, 25, 2),
    ("unit", 128, 128, 3, 12, 25, 1),
    ("unit", 128, 256, 2, 16, 33, 2),
    ("unit_nores", 3, 64, 4, 20, 25, 1),
]


@pytest.mark.parametrize("case", REAL_CASES, ids=["-".join(map(str, c)) for c in REAL_CASES])
def test_block_matches_oracle_real_widths(case):
    kind, cin, cout, NM, T, V, stride = case
    ref, ours = _pair(kind, cin, cout, V, stride, seed=cin * 31 + cout + T)
    x = formula.tensor((NM, cin, T, V), 5 + cin + cout, 1.0)
    To = T // stride if kind != "gcn" else T
    g = formula.tensor((NM, cout, To, V), 7 + cin + cout, 1.0)
    xr, yr, xo, yo = _run_pair(ref, ours, x, g)
    _compare(ref, ours, xr, yr, xo, yo, "-".join(map(str, case)))


def test_standalone_tcn_residual_conv_matches_oracle():
    import shiftgcn
    ref = mo.tcn(64, 128, kernel_size=1, stride=2)
    formula.fill_state(ref, seed=5)
    ours = shiftgcn.tcn(64, 128, kernel_size=1, stride=2).to(DEV)
    ours.load_state_dict(ref.state_dict())
    x = formula.tensor((3, 64, 21, 25), 9, 1.0)
    g = formula.tensor((3, 128, 11, 25), 10, 1.0)
    xr, yr, xo, yo = _run_pair(ref.train(), ours.train(), x, g)
    _compare(ref, ours, xr, yr, xo, yo, "tcn")


def test_eval_mode_forward_matches_oracle():
    ref, ours = _pair("unit", 64, 128, 25, 2, seed=77)
    ref.eval()
    ours.eval()
    x = formula.tensor((2, 64, 20, 25), 3, 1.0)
    with torch.no_grad():
        _rel_close(ours(x.to(DEV)).cpu(), ref(x), 2e-5, "eval unit")


@pytest.mark.parametrize("case", MODEL_CASES, ids=[c[0] for c in MODEL_CASES])
def test_model_matches_golden_fixture(golden, case):
    """Full Model at bs=2, T=300 (NTU: (2,3,300,25,2); MediaPipe: (2,3,300,33,1))."""
    import shiftgcn
    fx = golden("model_fixtures.npz")
    name, num_class, V, M, N, T = case
    m = shiftgcn.Model(num_class=num_class, num_point=V, num_person=M,
                       graph="graph.ntu_rgb_d.Graph")
    formula.fill_state(m, seed=97 + sum(map(ord, name)))
    m = m.to(DEV)
    x, labels = model_case_inputs(*case)
    m.eval()
    with torch.no_grad():   # running-statistics BatchNorms: well conditioned
        _rel_close(m(x.to(DEV)).cpu(), fx[f"model_{name}_logits_eval"], 1e-5, "eval logits")
    m.train()
    logits = m(x.to(DEV))
    loss = torch.nn.functional.cross_entropy(logits, labels.to(DEV))
    loss.backward()
    # train-mode logits and loss: no further from the reference's float64 run than 2x its
    # own fp32 run is (1e-5 floor), the bar the gradients are held to below
    l64 = torch.from_numpy(fx[f"model_{name}_logits_train64"]).double()
    l32 = torch.from_numpy(fx[f"model_{name}_logits_train"]).double()
    lo = logits.detach().cpu().double()
    sc = float(l64.abs().max())
    el_o, el_r = float((lo - l64).abs().max()) / sc, float((l32 - l64).abs().max()) / sc
    loss64 = float(torch.nn.functional.cross_entropy(l64, labels))
    ls_o = abs(float(loss) - loss64) / max(1.0, loss64)
    ls_r = abs(float(fx[f"model_{name}_loss"]) - loss64) / max(1.0, loss64)
    print(f"\n[{name} bs=2] train logits rel err vs fp64: HIP {el_o:.2e}, reference fp32 "
          f"{el_r:.2e}; loss {ls_o:.2e} vs {ls_r:.2e}")
    assert el_o <= max(2 * el_r, 1e-5), (el_o, el_r)
    assert ls_o <= max(2 * ls_r, 1e-5), (ls_o, ls_r)
    names = list(fx[f"model_{name}_grad_names"])
    params = dict(m.named_parameters())
    gnorm = np.array([float(params[n].grad.double().norm()) for n in names])
    # Model-level fp32 gradients through 10 BN units at bs=2 are ill-conditioned: the
    # reference's OWN fp32 CPU run differs from its float64 run by up to ~5e-3 relative in
    # grad norms (median ~1e-4) and flips the sign of 7-8 of 2816 ypos gradients.
    # Bar: the HIP path is as close to the float64 reference as the fp32 reference is
    # (median within 2x, worst parameter within 2x of the reference's worst).
    ref32, ref64 = fx[f"model_{name}_grad_norm"], fx[f"model_{name}_grad_norm64"]
    zero = np.array([n.endswith(("Linear_bias", "down.0.bias", "residual.conv.bias"))
                     for n in names])
    nz = ~zero & (ref64 > 0)      # xpos gradients are exactly 0 (x-shift is frozen)
    err_ours = np.abs(gnorm - ref64)[nz] / ref64[nz]
    err_ref = np.abs(ref32 - ref64)[nz] / ref64[nz]
    assert np.median(err_ours) <= 2 * np.median(err_ref) + 1e-5, (np.median(err_ours),
                                                                   np.median(err_ref))
    assert err_ours.max() <= 2 * err_ref.max(), (err_ours.max(), err_ref.max())
    assert np.all(gnorm[zero] < 1e-3)
    flips_ours = flips_ref = 0
    for n in names:
        if n.endswith("ypos"):
            s64 = np.sign(fx[f"model_{name}_grad64.{n}"])
            flips_ours += int((np.sign(params[n].grad.cpu().numpy()) != s64).sum())
            flips_ref += int((np.sign(fx[f"model_{name}_grad.{n}"]) != s64).sum())
    assert flips_ours <= 2 * flips_ref + 2, (flips_ours, flips_ref)


@pytest.mark.parametrize("kind,cin,cout,stride", [("unit", 64, 128, 2), ("unit", 64, 64, 1),
                                                  ("gcn", 3, 64, 1), ("tcn", 64, 64, 2)])
def test_eval_mode_backward_matches_oracle(kind, cin, cout, stride):
    """Backward through running-statistics BatchNorms (e.g. fine-tuning with frozen BN)."""
    ref, ours = _pair(kind, cin, cout, 25, stride, seed=5 + cin + cout)
    ref.eval()
    ours.eval()
    T = 12
    x = formula.tensor((2, cin, T, 25), 8 + cin, 1.0)
    To = T // stride if kind != "gcn" else T
    g = formula.tensor((2, cout, To, 25), 9 + cout, 1.0)
    xr, yr, xo, yo = _run_pair(ref, ours, x, g)
    _compare(ref, ours, xr, yr, xo, yo, f"eval-{kind}", train=False)


def test_model_backward_fusion_paths_taken(monkeypatch):
    """The cross-unit fusions are exercised by the model tests' numerics; this pins that
    they are actually taken: the next unit's gcn_dx_finish makes the bn2 backward partials
    of units l1, l2, l3, l6, l9 (successor without a conv residual), and the per-joint
    (gcn) partials of every unit — and, for l1 / l5 / l8, their down BatchNorm's — come out
    of the shift_in backward launch (sgcn_tshift_bwd_gbn), so only the 5 unit-tail reduce
    passes remain; every unit but l1 gets its gathered gcn input from the previous unit's
    tail launch (one standalone gather)."""
    import shiftgcn
    from shiftgcn import ops
    counts = {"reduce": 0, "gather": 0}
    real_reduce, real_gather = ops.bn_bwd_reduce, ops.gcn_gather

    def reduce(*a, **k):
        counts["reduce"] += 1
        return real_reduce(*a, **k)

    def gather(*a, **k):
        counts["gather"] += 1
        return real_gather(*a, **k)

    monkeypatch.setattr(ops, "bn_bwd_reduce", reduce)
    monkeypatch.setattr(ops, "gcn_gather", gather)
    m = shiftgcn.Model(num_class=60, num_point=25, num_person=2,
                       graph="graph.ntu_rgb_d.Graph").to(DEV).train()
    x = formula.tensor((2, 3, 16, 25, 2), 5, 1.0).to(DEV)
    m(x).sum().backward()
    torch.cuda.synchronize()
    assert counts["gather"] == 1, counts
    assert counts["reduce"] == 5, counts
