"""Pin the PyTorch-eager CPU model oracle to the reference modules (CPU; no GPU).

The fixtures were produced by the REFERENCE ``model/shift_gcn.py`` modules
(``tests/golden/gen_fixtures.py``); here the oracle restatement
(:mod:`oracle.model_oracle`) is run on the same deterministic weights and inputs.
"""
import numpy as np
import pytest
import torch

from oracle import model_oracle as mo
import formula
from gen_fixtures import (BLOCK_CASES, MODEL_CASES, block_case_inputs, build_block,
                          model_case_inputs)


@pytest.mark.parametrize("V", [25, 33])
@pytest.mark.parametrize("C", [3, 64, 128, 256])
def test_spatial_shift_indices_bit_exact(golden, V, C):
    fx = golden("shift_fixtures.npz")
    si = mo.spatial_shift_indices(V, C, +1)
    so_ = mo.spatial_shift_indices(V, C, -1)
    assert si.dtype == np.int64 and so_.dtype == np.int64
    assert np.array_equal(si, fx[f"shift_in_V{V}_C{C}"])
    assert np.array_equal(so_, fx[f"shift_out_V{V}_C{C}"])
    # both are permutations
    assert np.array_equal(np.sort(si), np.arange(V * C))
    assert np.array_equal(np.sort(so_), np.arange(V * C))



@pytest.mark.parametrize("case", BLOCK_CASES, ids=[c[0] for c in BLOCK_CASES])
def test_block_matches_reference(golden, case):
    fx = golden("block_fixtures.npz")
    name, kind, cin, cout, NM, T, V, stride = case
    m = build_block(mo, kind, cin, cout, V, stride)
    formula.fill_state(m, seed=31 + sum(map(ord, name)))
    m.train()
    x, g = block_case_inputs(name, kind, cin, cout, NM, T, V, stride)
    xr = x.clone().requires_grad_(True)
    y = m(xr)
    y.backward(g)
    np.testing.assert_allclose(y.detach().numpy(), fx[f"blk_{name}_out"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(xr.grad.numpy(), fx[f"blk_{name}_gx"], rtol=1e-5, atol=1e-5)
    for pn, p in m.named_parameters():
        key = f"blk_{name}_grad.{pn}"
        if p.grad is None:
            assert key not in fx.files
            continue
        ref = fx[key]
        if pn.endswith(("xpos", "ypos")):
            assert np.array_equal(p.grad.numpy(), ref), pn
        else:
            np.testing.assert_allclose(p.grad.numpy(), ref, rtol=1e-4, atol=1e-4, err_msg=pn)
    for bn, b in m.named_buffers():
        if b.dtype.is_floating_point:
            np.testing.assert_allclose(b.numpy(), fx[f"blk_{name}_buf.{bn}"], rtol=1e-5,
                                       atol=1e-6, err_msg=bn)


@pytest.mark.parametrize("case", MODEL_CASES, ids=[c[0] for c in MODEL_CASES])
def test_model_matches_reference(golden, case):
    fx = golden("model_fixtures.npz")
    name, num_class, V, M, N, T = case
    torch.set_num_threads(max(1, min(8, torch.get_num_threads())))
    m = mo.Model(num_class=num_class, num_point=V, num_person=M, graph="unused")
    formula.fill_state(m, seed=97 + sum(map(ord, name)))
    x, labels = model_case_inputs(name, num_class, V, M, N, T)
    m.eval()
    with torch.no_grad():
        np.testing.assert_allclose(m(x).numpy(), fx[f"model_{name}_logits_eval"],
                                   rtol=1e-4, atol=1e-4)
    m.train()
    logits = m(x)
    loss = torch.nn.functional.cross_entropy(logits, labels)
    loss.backward()
    np.testing.assert_allclose(logits.detach().numpy(), fx[f"model_{name}_logits_train"],
                               rtol=1e-4, atol=1e-4)
    names = list(fx[f"model_{name}_grad_names"])
    params = dict(m.named_parameters())
    assert names == [pn for pn, p in m.named_parameters() if p.grad is not None]
    gsum = np.array([float(params[n].grad.double().sum()) for n in names])
    gnorm = np.array([float(params[n].grad.double().norm()) for n in names])
    np.testing.assert_allclose(gnorm, fx[f"model_{name}_grad_norm"], rtol=1e-3, atol=1e-6)
    np.testing.assert_allclose(gsum, fx[f"model_{name}_grad_sum"], rtol=1e-3,
                               atol=1e-3 * np.abs(fx[f"model_{name}_grad_sum"]).max())
    for n in names:
        if n.endswith(("xpos", "ypos")):
            assert np.array_equal(params[n].grad.numpy(), fx[f"model_{name}_grad.{n}"]), n
