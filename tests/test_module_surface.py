"""Drop-in surface (CPU): same constructor signatures, state_dict keys, shapes and dtypes
as the reference modules (pinned through the oracle, itself pinned to the reference)."""
import inspect

import pytest
import torch

import shiftgcn
from oracle import model_oracle as mo


@pytest.mark.parametrize("name", ["tcn", "Shift_tcn", "Shift_gcn", "TCN_GCN_unit", "Model"])
def test_constructor_signatures(name):
    a = inspect.signature(getattr(shiftgcn, name).__init__)
    b = inspect.signature(getattr(mo, name).__init__)
    assert list(a.parameters) == list(b.parameters)
    for k in a.parameters:
        assert a.parameters[k].default == b.parameters[k].default, k


def test_shift_signature():
    from oracle.model_oracle import Shift as OShift
    a = inspect.signature(shiftgcn.Shift.__init__).parameters
    assert list(a)[:4] == list(inspect.signature(OShift.__init__).parameters)


@pytest.mark.parametrize("V,M,nc,nparams", [(25, 2, 60, 693107), (33, 1, 2, 709867)])
def test_state_dict_matches_reference_layout(V, M, nc, nparams):
    ours = shiftgcn.Model(num_class=nc, num_point=V, num_person=M, graph="graph.ntu_rgb_d.Graph")
    ref = mo.Model(num_class=nc, num_point=V, num_person=M, graph="unused")
    sa, sb = ours.state_dict(), ref.state_dict()
    assert list(sa) == list(sb)
    for k in sa:
        assert sa[k].shape == sb[k].shape and sa[k].dtype == sb[k].dtype, k
    assert torch.equal(sa["l1.gcn1.shift_in"], sb["l1.gcn1.shift_in"])
    assert torch.equal(sa["l8.gcn1.shift_out"], sb["l8.gcn1.shift_out"])
    n = sum(p.numel() for p in ours.parameters() if p.requires_grad)
    assert n == nparams
    # reference checkpoints load unchanged
    ours.load_state_dict(sb)


def test_graph_strings():
    for g in ("graph.ntu_rgb_d.Graph", "graph.mediapipe_pose.Graph",
              "shiftgcn.graph.ntu_rgb_d.Graph"):
        m = shiftgcn.Model(num_point=25, graph=g)
        assert m.graph.A.shape[0] == 3
