"""Autograd robustness of the fused blocks (shiftgcn/fused.py `_BlockFunction`) and the
cross-unit backward fusions' invariants.

* an in-place op on a block's output (or input) between forward and backward raises
  autograd's version-counter error instead of corrupting the ReLU-mask / BN backward;
* a second backward through the same graph raises a clear RuntimeError;
* a unit chain where the second unit has a gcn ``down`` conv and NO residual (so the
  previous unit's bn2 backward partials must NOT be taken from the second unit's
  gcn_dx_finish, whose dx is still missing the down-conv gradient) matches the oracle.
"""
import pytest
import torch

import formula
from oracle import model_oracle as mo
from test_gpu_blocks import _compare

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _unit(cin=64, cout=64, stride=1, residual=True):
    import shiftgcn
    u = shiftgcn.TCN_GCN_unit(cin, cout, None, stride=stride, residual=residual, num_point=25)
    formula.fill_state(u, seed=cin + cout)
    return u.to(DEV).train()


def test_inplace_on_block_output_raises():
    u = _unit()
    x = formula.tensor((2, 64, 12, 25), 1, 1.0).to(DEV).requires_grad_(True)
    y = u(x)
    y.add_(1.0)
    with pytest.raises(RuntimeError, match="inplace"):
        y.sum().backward()


def test_inplace_on_block_input_raises():
    u = _unit()
    x0 = formula.tensor((2, 64, 12, 25), 1, 1.0).to(DEV).requires_grad_(True)
    x = x0 * 1.0
    y = u(x)
    x.mul_(2.0)
    with pytest.raises(RuntimeError, match="inplace"):
        y.sum().backward()


def test_second_backward_raises_clear_error():
    u = _unit()
    x = formula.tensor((2, 64, 12, 25), 1, 1.0).to(DEV).requires_grad_(True)
    y = u(x)
    y.sum().backward(retain_graph=True)
    with pytest.raises(RuntimeError, match="second time"):
        y.sum().backward()


def test_chain_identity_then_down_noresidual_matches_oracle():
    """l(64->64, identity residual) followed by (64->128, residual=False): the second unit's
    gcn has a down conv, so its gcn_dx_finish must not make the first unit's bn2 partials."""
    import shiftgcn
    from shiftgcn.shift_gcn import linked_units

    ref = torch.nn.Sequential(mo.TCN_GCN_unit(64, 64, None, num_point=25),
                              mo.TCN_GCN_unit(64, 128, None, residual=False, num_point=25))
    formula.fill_state(ref, seed=41)
    ours = torch.nn.Sequential(shiftgcn.TCN_GCN_unit(64, 64, None, num_point=25),
                               shiftgcn.TCN_GCN_unit(64, 128, None, residual=False,
                                                     num_point=25)).to(DEV)
    ours.load_state_dict(ref.state_dict())
    ref.train()
    ours.train()
    x = formula.tensor((3, 64, 16, 25), 42, 1.0)
    g = formula.tensor((3, 128, 16, 25), 43, 1.0)
    xr = x.clone().requires_grad_(True)
    yr = ref(xr)
    yr.backward(g)
    xo = x.to(DEV).requires_grad_(True)
    with linked_units(list(ours)):
        yo = ours(xo)
    yo.backward(g.to(DEV))
    torch.cuda.synchronize()
    _compare(ref, ours, xr, yr, xo, yo, "chain")
