"""FusedSGD (sgcn_sgd_step: every parameter updated in one launch) against torch.optim.SGD,
the reference harness's optimizer (main.py:301-322, 414): same parameters and momentum
buffers after several steps, within fp32 rounding (the native update may fuse a
multiply-add that torch's foreach kernels round twice), for the reference's settings
(nesterov, momentum 0.9, per-group weight decay incl. 0) and the other supported ones."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _params(seed):
    g = torch.Generator().manual_seed(seed)
    shapes = [(64, 64), (256,), (3, 64, 1, 1), (5000,), (1, 25, 64), (7,)]
    return [torch.randn(s, generator=g).to(DEV) for s in shapes]


def _groups(ps, lr):
    return [{"params": ps[:2], "lr": lr, "weight_decay": 1e-3},
            {"params": ps[2:4], "lr": lr, "weight_decay": 0.0},
            {"params": ps[4:], "lr": lr, "weight_decay": 1e-4}]


def _rel(a, b):
    return float((a - b).abs().max()) / (float(b.abs().max()) + 1e-30)


@pytest.mark.parametrize("momentum,nesterov", [(0.9, True), (0.9, False), (0.0, False)])
def test_fused_sgd_matches_torch(momentum, nesterov):
    from shiftgcn.train import FusedSGD
    ref = [p.clone().requires_grad_(True) for p in _params(1)]
    ours = [p.clone().requires_grad_(True) for p in _params(1)]
    o_ref = torch.optim.SGD(_groups(ref, 0.1), lr=0.1, momentum=momentum, nesterov=nesterov)
    o_ours = FusedSGD(_groups(ours, 0.1), lr=0.1, momentum=momentum, nesterov=nesterov)
    g = torch.Generator().manual_seed(7)
    for step in range(4):
        grads = [torch.randn(p.shape, generator=g).to(DEV) for p in ref]
        for ps in (ref, ours):
            for p, gr in zip(ps, grads):
                p.grad = gr.clone()
        if step == 2:   # the LR schedule rewrites every group's lr between steps
            for o in (o_ref, o_ours):
                for grp in o.param_groups:
                    grp["lr"] = 0.01
        o_ref.step()
        o_ours.step()
    torch.cuda.synchronize()
    for a, b in zip(ours, ref):
        assert _rel(a.detach(), b.detach()) < 1e-6
    if momentum:
        for a, b in zip(ours, ref):
            assert _rel(o_ours.state[a]["momentum_buffer"], o_ref.state[b]["momentum_buffer"]) < 1e-6


def test_fused_sgd_state_dict_round_trip():
    """A stock optimizer's state loads into FusedSGD (and back) and the next step agrees."""
    from shiftgcn.train import FusedSGD
    ref = [p.clone().requires_grad_(True) for p in _params(3)]
    ours = [p.clone().requires_grad_(True) for p in _params(3)]
    o_ref = torch.optim.SGD(_groups(ref, 0.1), lr=0.1, momentum=0.9, nesterov=True)
    g = torch.Generator().manual_seed(9)
    grads = [torch.randn(p.shape, generator=g).to(DEV) for p in ref]
    for p, gr in zip(ref, grads):
        p.grad = gr.clone()
    o_ref.step()
    with torch.no_grad():
        for a, b in zip(ours, ref):
            a.copy_(b)
    o_ours = FusedSGD(_groups(ours, 0.1), lr=0.1, momentum=0.9, nesterov=True)
    # (a deep copy: load_state_dict keeps a same-device buffer as the SAME tensor, which
    # o_ref's next step would then update for both optimizers)
    o_ours.load_state_dict(copy.deepcopy(o_ref.state_dict()))
    grads = [torch.randn(p.shape, generator=g).to(DEV) for p in ref]
    for ps in (ref, ours):
        for p, gr in zip(ps, grads):
            p.grad = gr.clone()
    o_ref.step()
    o_ours.step()
    torch.cuda.synchronize()
    for a, b in zip(ours, ref):
        assert _rel(a.detach(), b.detach()) < 1e-6
    o_back = torch.optim.SGD(_groups(ref, 0.1), lr=0.1, momentum=0.9, nesterov=True)
    o_back.load_state_dict(o_ours.state_dict())


def test_model_training_step_with_fused_sgd():
    """One reference training step of the model: the fused optimizer and torch's SGD leave
    the same parameters (the same gradients in, fp32 rounding apart; one step only: a second
    step's shift-position gradients are signs of near-tied sums)."""
    import shiftgcn
    from shiftgcn import train
    m1 = shiftgcn.Model(num_class=60, num_point=25, num_person=2,
                        graph="graph.ntu_rgb_d.Graph").to(DEV).train()
    m2 = copy.deepcopy(m1)
    o1 = train.build_optimizer(m1, base_lr=0.1, fused=False)
    o2 = train.build_optimizer(m2, base_lr=0.1, fused=True)
    assert isinstance(o2, train.FusedSGD)
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 3, 16, 25, 2, generator=g).to(DEV)
    y = torch.randint(0, 60, (2,), generator=g).to(DEV)
    train.train_step(m1, o1, x, y)
    train.train_step(m2, o2, x, y)
    torch.cuda.synchronize()
    for (n, a), (_, b) in zip(m2.named_parameters(), m1.named_parameters()):
        assert _rel(a.detach(), b.detach()) < 1e-5, n


def test_fused_sgd_host_momentum_buffer_is_not_passed_to_the_kernel():
    """Optimizer state loaded while the parameters were on the host keeps its momentum
    buffers there after the parameters move to the GPU. The native update must not take
    those host pointers (the kernel would dereference them); FusedSGD then behaves exactly
    like torch.optim.SGD (which raises, or updates identically)."""
    from shiftgcn.train import FusedSGD

    def run(cls):
        g = torch.Generator().manual_seed(11)
        ps = [torch.nn.Parameter(torch.randn(s, generator=g)) for s in ((64, 8), (33,))]
        o = cls(ps, lr=0.1, momentum=0.9, nesterov=True)
        for p in ps:
            p.grad = torch.randn(p.shape, generator=g)
        o.step()                               # host-side momentum buffers
        for p in ps:                           # the parameters move, the state does not
            p.data = p.data.to(DEV)
            p.grad = torch.randn(p.shape, generator=g).to(DEV)
        assert all(o.state[p]["momentum_buffer"].device.type == "cpu" for p in ps)
        try:
            o.step()
        except RuntimeError as e:
            return ("raised", type(e))
        torch.cuda.synchronize()
        return ("ok", [p.detach().cpu() for p in ps])

    ref, ours = run(torch.optim.SGD), run(FusedSGD)
    assert ref[0] == ours[0]
    if ref[0] == "ok":
        for a, b in zip(ours[1], ref[1]):
            assert torch.equal(a, b)


def test_fused_sgd_deferred_grad_scale_matches_multiply_then_step():
    """sgcn_sgd_step flags bit 1: grad *= s inside the update (GradAllReduce's deferred
    DataParallel 1/world), stored back: same parameters, buffers and .grad as a separate
    multiply followed by the step, bit for bit."""
    from shiftgcn.train import FusedSGD
    a = [p.clone().requires_grad_(True) for p in _params(21)]
    b = [p.clone().requires_grad_(True) for p in _params(21)]
    oa = FusedSGD(_groups(a, 0.1), lr=0.1, momentum=0.9, nesterov=True)
    ob = FusedSGD(_groups(b, 0.1), lr=0.1, momentum=0.9, nesterov=True)
    g = torch.Generator().manual_seed(22)
    scales = [0.125, 1.0 / 3.0, 0.5, 1.0, 0.25, 1.0 / 7.0]
    for _ in range(3):
        grads = [torch.randn(p.shape, generator=g).to(DEV) for p in a]
        for ps in (a, b):
            for p, gr in zip(ps, grads):
                p.grad = gr.clone()
        with torch.no_grad():
            for p, s in zip(b, scales):
                p.grad.mul_(s)
        oa.defer_grad_scale([(p, s) for p, s in zip(a, scales) if s != 1.0])
        oa.step()
        ob.step()
    torch.cuda.synchronize()
    for p, q in zip(a, b):
        assert torch.equal(p, q)
        assert torch.equal(p.grad, q.grad)
        assert torch.equal(oa.state[p]["momentum_buffer"], ob.state[q]["momentum_buffer"])
