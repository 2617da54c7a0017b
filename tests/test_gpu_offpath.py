"""Weight gradients on the side stream (fused._OffPath, linked units in Model.forward).

* The whole model's gradients and BatchNorm running statistics are bit-identical with the
  side stream on and off (every kernel is deterministic, so any race would show up as a
  mismatch), over two consecutive training steps (the second one reuses freed memory).
* Autograd takes the side-stream gradient tensors as they are: each weight gradient
  produced by a contraction IS the parameter's ``.grad`` afterwards (no clone launched on
  the current stream before the join).
* ``.grad`` already set (gradient accumulation), a regulariser term in the loss, a
  parameter tied across two units, the data-parallel bucket, ``torch.autograd.grad`` and
  ``backward(inputs=...)``: the deferred gradients (never handed to autograd, accumulated
  into ``.grad`` at the end of the backward, ``fused._finish``) give exactly the in-order
  path's gradients.
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


def test_post_accumulate_grad_hook_sees_finished_gradient():
    """a ``register_post_accumulate_grad_hook`` on a Feature_Mask and on
    a ypos reads ``.grad`` right after AccumulateGrad: those units must neither defer the
    gradient write (side stream / end-of-backward batch) nor hand out an unwritten tensor.
    The hooks see the finished gradients and the step equals the in-order path bit for
    bit."""
    from shiftgcn import fused
    dev = torch.device("cuda:0")
    x = formula.tensor((4, 3, 64, 25, 2), 45, 1.0).to(dev)
    y = torch.tensor([5, 6, 7, 8], device=dev)
    seen, grads = {}, {}
    for mode in (0, 1):
        old, oldb = fused.ASYNC_DW, fused.BATCH_SIDE
        fused.ASYNC_DW = fused.BATCH_SIDE = mode
        try:
            m = _model(dev)
            for name in ("l3.gcn1.Feature_Mask", "l6.tcn1.shift_in.ypos",
                         "l2.gcn1.Feature_Mask"):
                p = m.get_parameter(name)
                p.register_post_accumulate_grad_hook(
                    lambda t, k=(mode, name): seen.__setitem__(k, t.grad.detach().clone()))
            for p in m.parameters():
                p.grad = None
            torch.nn.functional.cross_entropy(m(x), y).backward()
            torch.cuda.synchronize()
            grads[mode] = {n: p.grad.cpu() for n, p in m.named_parameters()
                           if p.grad is not None}
            for name in ("l3.gcn1.Feature_Mask", "l6.tcn1.shift_in.ypos",
                         "l2.gcn1.Feature_Mask"):   # the hook saw the final .grad
                assert torch.equal(seen[(mode, name)].cpu(), grads[mode][name]), name
        finally:
            fused.ASYNC_DW, fused.BATCH_SIDE = old, oldb
    for k in grads[0]:
        assert torch.equal(grads[0][k], grads[1][k]), k
    assert float(grads[1]["l3.gcn1.Feature_Mask"].abs().max()) > 0


def _twice_grads(dev, async_dw, one_graph, slots=False):
    """Gradients of CE(m(a)) + CE(m(b)): summed in ONE backward (the model used twice in
    one graph), or as two backward passes accumulating into .grad."""
    from shiftgcn import fused
    from shiftgcn.dist import GradAllReduce
    old = fused.ASYNC_DW
    fused.ASYNC_DW = async_dw
    ga = None
    try:
        m = _model(dev)
        if slots:   # gradient bucket slots registered (the data-parallel step)
            ga = GradAllReduce(m)
        a = formula.tensor((4, 3, 64, 25, 2), 46, 1.0).to(dev)
        b = formula.tensor((4, 3, 64, 25, 2), 47, 1.0).to(dev)
        ya = torch.tensor([1, 2, 3, 4], device=dev)
        yb = torch.tensor([9, 8, 7, 6], device=dev)
        for p in m.parameters():
            p.grad = None
        ce = torch.nn.functional.cross_entropy
        if one_graph:
            (ce(m(a), ya) + ce(m(b), yb)).backward()
        else:
            ce(m(a), ya).backward()
            ce(m(b), yb).backward()
        if ga is not None:
            ga()
        torch.cuda.synchronize()
        return {n: p.grad.detach().cpu().clone() for n, p in m.named_parameters()
                if p.grad is not None}
    finally:
        fused.ASYNC_DW = old
        if ga is not None:
            ga.close()


def test_model_used_twice_in_one_graph():
    """a parameter with two gradient contributions in one backward.
    The deferred writes (side stream, end-of-backward finalizes) and the gradient bucket
    slots must not hand autograd a tensor it sums before it is written, nor the same slot
    twice: one backward over model(a) + model(b) equals two accumulating backward passes,
    with and without the side stream and with the data-parallel bucket registered."""
    import socket

    import torch.distributed as dist
    dev = torch.device("cuda:0")
    ref = _twice_grads(dev, 0, one_graph=False)
    for async_dw in (1, 0):
        got = _twice_grads(dev, async_dw, one_graph=True)
        assert got.keys() == ref.keys() and len(got) > 100
        for n in ref:
            torch.testing.assert_close(got[n], ref[n], rtol=1e-6, atol=1e-7, msg=n)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0,
                            world_size=1)
    try:
        got = _twice_grads(dev, 1, one_graph=True, slots=True)
        for n in ref:
            torch.testing.assert_close(got[n], ref[n], rtol=1e-6, atol=1e-7, msg=n)
    finally:
        dist.destroy_process_group()


def test_two_autograd_grad_calls_get_distinct_slots():
    """two torch.autograd.grad calls while the bucket is registered
    return tensors that do not alias each other (a slot goes to one gradient per backward)."""
    import shiftgcn
    from shiftgcn import ops
    dev = torch.device("cuda:0")
    u = shiftgcn.TCN_GCN_unit(64, 64, None, num_point=25)
    formula.fill_state(u, seed=8)
    u = u.to(dev).train()
    ps = [p for p in u.parameters() if p.requires_grad]
    x1 = formula.tensor((2, 64, 16, 25), 50, 1.0).to(dev)
    x2 = formula.tensor((2, 64, 16, 25), 51, 1.0).to(dev)
    # references without a bucket (training-mode outputs use batch statistics, so the
    # running-statistics updates between calls change nothing)
    ref1 = [t.clone() for t in torch.autograd.grad(u(x1).square().sum(), ps)]
    ref2 = [t.clone() for t in torch.autograd.grad(u(x2).square().sum(), ps)]
    flat = torch.zeros(sum(p.numel() for p in ps), device=dev)
    ops.register_grad_slots([(str(i), p) for i, p in enumerate(ps)], flat)
    try:
        g1 = torch.autograd.grad(u(x1).square().sum(), ps)
        g2 = torch.autograd.grad(u(x2).square().sum(), ps)
        torch.cuda.synchronize()
        lo, hi = flat.data_ptr(), flat.data_ptr() + 4 * flat.numel()
        assert all(lo <= a.data_ptr() < hi for a in g1)          # the first got the slots
        assert not any(lo <= b.data_ptr() < hi for b in g2)      # the second fresh memory
        for a, r in zip(g1, ref1):   # ... and did not overwrite the first one's results
            assert torch.equal(a, r)
        for b, r in zip(g2, ref2):
            assert torch.equal(b, r)
    finally:
        ops.unregister_grad_slots(ps)
        ops.release_grad_slots(ps)


_REG = ("Linear_weight", "Feature_Mask", "ypos", "conv.weight", "temporal_linear.weight",
        "down.0.weight")


def _extra_grads(dev, mode, variant, slots=False):
    """Gradients of one step whose parameters also get a contribution from OUTSIDE their
    unit: ``l2`` = CE + 1e-3 * sum ||p||^2 over the Linear / mask / ypos / conv weights,
    ``tied`` = l3's Linear_weight IS l2's, ``tied_l2`` = both. ``mode`` 1 = side stream and
    deferred finalizes, 0 = everything in order."""
    from shiftgcn import fused
    from shiftgcn.dist import GradAllReduce
    old = fused.ASYNC_DW, fused.BATCH_SIDE
    fused.ASYNC_DW = fused.BATCH_SIDE = mode
    ga = None
    try:
        m = _model(dev)
        if variant.startswith("tied"):
            m.l3.gcn1.Linear_weight = m.l2.gcn1.Linear_weight
        if slots:
            ga = GradAllReduce(m)
        x = formula.tensor((4, 3, 64, 25, 2), 48, 1.0).to(dev)
        y = torch.tensor([0, 4, 2, 9], device=dev)
        for p in m.parameters():
            p.grad = None
        loss = torch.nn.functional.cross_entropy(m(x), y)
        if variant.endswith("l2"):
            reg = [p for n, p in m.named_parameters() if n.endswith(_REG)]
            assert len(reg) > 40
            loss = loss + 1e-3 * sum(p.square().sum() for p in reg)
        loss.backward()
        if ga is not None:
            ga()
            # every gradient is (still) its bucket slot
            assert all(ops_is_slot(p) for _, p in ga.named)
        torch.cuda.synchronize()
        return {n: p.grad.detach().cpu().clone() for n, p in m.named_parameters()
                if p.grad is not None}
    finally:
        fused.ASYNC_DW, fused.BATCH_SIDE = old
        if ga is not None:
            ga.close()


def ops_is_slot(p):
    from shiftgcn import ops
    return p.grad is not None and ops.is_grad_slot(p, p.grad)


@pytest.fixture
def gloo_world1():
    import socket

    import torch.distributed as dist
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0,
                            world_size=1)
    try:
        yield
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("variant", ["l2", "tied", "tied_l2"])
def test_gradient_from_outside_the_unit_bit_identical(variant):
    """a parameter whose gradient also comes from outside its
    unit (a loss regulariser, a tied parameter). The side stream and the deferred finalizes
    must give the in-order path's gradients bit for bit."""
    dev = torch.device("cuda:0")
    ref = _extra_grads(dev, 0, variant)
    got = _extra_grads(dev, 1, variant)
    assert got.keys() == ref.keys() and len(got) > 100
    for n in ref:
        assert torch.equal(got[n], ref[n]), n
    if variant.endswith("l2"):   # the regulariser really reached those gradients
        plain = _extra_grads(dev, 0, "tied" if variant == "tied_l2" else "none")
        assert not torch.equal(plain["l2.gcn1.Feature_Mask"], ref["l2.gcn1.Feature_Mask"])


@pytest.mark.parametrize("variant", ["l2", "tied_l2"])
def test_gradient_from_outside_the_unit_with_bucket(variant, gloo_world1):
    """The same with the data-parallel gradient bucket registered (GradAllReduce, world 1):
    identical gradients, and every .grad is its bucket slot after the reduction."""
    dev = torch.device("cuda:0")
    ref = _extra_grads(dev, 0, variant, slots=True)
    got = _extra_grads(dev, 1, variant, slots=True)
    assert got.keys() == ref.keys()
    for n in ref:
        assert torch.equal(got[n], ref[n]), n
    plain = _extra_grads(dev, 0, variant)
    for n in ref:
        assert torch.equal(got[n], plain[n]), n


def test_autograd_grad_and_backward_inputs_in_order():
    """``torch.autograd.grad`` over some parameters and ``backward(inputs=...)`` with the side
    stream on: the units whose gradients are captured or not accumulated run in order, and
    the results equal the in-order path's."""
    from shiftgcn import fused
    dev = torch.device("cuda:0")
    x = formula.tensor((4, 3, 64, 25, 2), 49, 1.0).to(dev)
    y = torch.tensor([1, 1, 2, 3], device=dev)
    names = ("l4.gcn1.Linear_weight", "l7.tcn1.shift_in.ypos", "l2.gcn1.Feature_Mask",
             "l9.tcn1.temporal_linear.weight")
    res = {}
    for mode in (0, 1):
        old = fused.ASYNC_DW, fused.BATCH_SIDE
        fused.ASYNC_DW = fused.BATCH_SIDE = mode
        try:
            m = _model(dev)
            ps = [m.get_parameter(n) for n in names]
            g = torch.autograd.grad(torch.nn.functional.cross_entropy(m(x), y), ps)
            for p in m.parameters():
                p.grad = None
            torch.nn.functional.cross_entropy(m(x), y).backward(inputs=ps[:2])
            torch.cuda.synchronize()
            assert all(p.grad is None for n, p in m.named_parameters()
                       if n not in names[:2])
            res[mode] = ([t.cpu() for t in g], [p.grad.cpu() for p in ps[:2]])
        finally:
            fused.ASYNC_DW, fused.BATCH_SIDE = old
        assert not fused._TASKS
    for a, b in zip(res[0][0] + res[0][1], res[1][0] + res[1][1]):
        assert torch.equal(a, b)
