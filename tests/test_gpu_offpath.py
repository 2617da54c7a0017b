"""Weight gradients on the side stream (fused._OffPath, linked units in Model.forward).

* The whole model's gradients and BatchNorm running statistics are bit-identical with the
  side stream on and off (every kernel is deterministic, so any race would show up as a
  mismatch), over two consecutive training steps (the second one reuses freed memory).
* Autograd takes the side-stream gradient tensors as they are: each weight gradient
  produced by a contraction IS the parameter's ``.grad`` afterwards (no clone launched on
  the current stream before the join).
* ``.grad`` already set (gradient accumulation) falls back to the in-order path, and the
  accumulated result equals two synchronous backward passes.
"""
import pytest
import torch

import formula

pytestmark = pytest.mark.gpu


def _model(dev):
    import shiftgcn
    m = shiftgcn.Model(num_class=10, num_point=25, num_person=2, graph="graph.ntu_rgb_d.Graph")
    formula.fill_state(m, seed=5)
    return m.to(dev).train()


def _step(m, x, y):
    out = m(x)
    loss = torch.nn.functional.cross_entropy(out, y)
    for p in m.parameters():
        p.grad = None
    loss.backward()
    return loss.detach()


def _run(async_dw, steps=2):
    from shiftgcn import fused
    dev = torch.device("cuda:0")
    old = fused.ASYNC_DW
    fused.ASYNC_DW = async_dw
    try:
        m = _model(dev)
        res = []
        for k in range(steps):
            x = formula.tensor((4, 3, 64, 25, 2), 40 + k, 1.0).to(dev)
            y = torch.tensor([1, 3, 5, 7], device=dev)
            loss = _step(m, x, y)
            torch.cuda.synchronize()
            res.append((loss.cpu(), {n: p.grad.detach().cpu().clone()
                                     for n, p in m.named_parameters() if p.grad is not None},
                        {n: b.detach().cpu().clone() for n, b in m.named_buffers()}))
        return res
    finally:
        fused.ASYNC_DW = old


def test_side_stream_gradients_bit_identical():
    a, b = _run(1), _run(0)
    for (la, ga, ba), (lb, gb, bb) in zip(a, b):
        assert torch.equal(la, lb)
        assert ga.keys() == gb.keys() and len(ga) > 100
        for n in ga:
            assert torch.equal(ga[n], gb[n]), n
        for n in ba:
            assert torch.equal(ba[n], bb[n]), n


@pytest.mark.parametrize("tail", [0, 1, 2])
def test_end_of_backward_variants_bit_identical(tail, monkeypatch):
    """SGCN_TAIL_MAIN (the deferred finalizes / the last unit's weight gradients on the
    main stream; the default is 3) and the once-per-backward join: same results."""
    from shiftgcn import fused
    monkeypatch.setattr(fused, "TAIL_MAIN", tail)
    a = _run(1)
    monkeypatch.setattr(fused, "TAIL_MAIN", 3)
    b = _run(0)
    for (la, ga, ba), (lb, gb, bb) in zip(a, b):
        assert torch.equal(la, lb)
        assert ga.keys() == gb.keys()
        for n in ga:
            assert torch.equal(ga[n], gb[n]), n
        for n in ba:
            assert torch.equal(ba[n], bb[n]), n


def test_side_stream_gradients_are_taken_not_copied(monkeypatch):
    from shiftgcn import fused, ops
    dev = torch.device("cuda:0")
    ptrs = []
    real = ops.pw_dw

    def rec(g, x, dw, *a, **k):
        ptrs.append(dw.data_ptr())
        return real(g, x, dw, *a, **k)

    monkeypatch.setattr(ops, "pw_dw", rec)
    monkeypatch.setattr(fused, "ASYNC_DW", 1)
    m = _model(dev)
    x = formula.tensor((4, 3, 64, 25, 2), 41, 1.0).to(dev)
    _step(m, x, torch.tensor([0, 1, 2, 3], device=dev))
    torch.cuda.synchronize()
    grads = {p.grad.data_ptr() for p in m.parameters() if p.grad is not None}
    assert len(ptrs) >= 20
    assert all(q in grads for q in ptrs)


def test_existing_grad_accumulates_in_order():
    from shiftgcn import fused
    dev = torch.device("cuda:0")
    x = formula.tensor((4, 3, 64, 25, 2), 42, 1.0).to(dev)
    y = torch.tensor([2, 4, 6, 8], device=dev)
    ref = {}
    for mode in (0, 1):
        old = fused.ASYNC_DW
        fused.ASYNC_DW = mode
        try:
            m = _model(dev)
            for p in m.parameters():
                p.grad = None
            for _ in range(2):       # the second backward accumulates into .grad
                torch.nn.functional.cross_entropy(m(x), y).backward()
            torch.cuda.synchronize()
            ref[mode] = {n: p.grad.cpu() for n, p in m.named_parameters() if p.grad is not None}
        finally:
            fused.ASYNC_DW = old
    for n in ref[0]:
        assert torch.equal(ref[0][n], ref[1][n]), n


def test_parameter_hook_sees_finished_gradient():
    """A gradient hook on a weight reads it during the backward: that unit must not use
    the side stream (the hook would otherwise see an unwritten tensor)."""
    from shiftgcn import fused
    dev = torch.device("cuda:0")
    x = formula.tensor((4, 3, 64, 25, 2), 43, 1.0).to(dev)
    y = torch.tensor([1, 2, 3, 4], device=dev)
    seen = {}
    for mode in (0, 1):
        old = fused.ASYNC_DW
        fused.ASYNC_DW = mode
        try:
            m = _model(dev)
            w = m.l9.tcn1.temporal_linear.weight
            w.register_hook(lambda g, mode=mode: seen.__setitem__(mode, g.detach().clone()))
            torch.nn.functional.cross_entropy(m(x), y).backward()
            torch.cuda.synchronize()
        finally:
            fused.ASYNC_DW = old
    assert torch.equal(seen[0], seen[1])



def test_create_graph_backward_stays_in_order():
    """backward(create_graph=True) runs the units' backward with grad mode on, where
    AccumulateGrad clones a gradient on the current stream instead of taking it: the side
    stream must not be used, and the gradients equal a plain backward's."""
    from shiftgcn import fused
    dev = torch.device("cuda:0")
    x = formula.tensor((4, 3, 64, 25, 2), 44, 1.0).to(dev)
    y = torch.tensor([3, 1, 4, 1], device=dev)
    res = {}
    for mode, cg in ((0, False), (1, True)):
        old = fused.ASYNC_DW
        fused.ASYNC_DW = mode
        try:
            m = _model(dev)
            for p in m.parameters():
                p.grad = None
            torch.nn.functional.cross_entropy(m(x), y).backward(create_graph=cg)
            torch.cuda.synchronize()
            res[mode] = {n: p.grad.detach().cpu() for n, p in m.named_parameters()
                         if p.grad is not None}
        finally:
            fused.ASYNC_DW = old
    assert res[0].keys() == res[1].keys() and len(res[0]) > 100
    for n in res[0]:
        assert torch.equal(res[0][n], res[1][n]), n
