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
