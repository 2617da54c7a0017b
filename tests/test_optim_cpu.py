"""FusedSGD host logic without a GPU: CPU parameters take torch's own SGD step (the native
update is device-only), so the optimizer stays a drop-in for torch.optim.SGD."""
import torch


def test_fused_sgd_cpu_falls_back_to_torch():
    from shiftgcn.train import FusedSGD
    g = torch.Generator().manual_seed(0)
    a = [torch.randn(5, 3, generator=g).requires_grad_(True) for _ in range(2)]
    b = [p.detach().clone().requires_grad_(True) for p in a]
    oa = FusedSGD([{"params": a[:1], "weight_decay": 1e-3}, {"params": a[1:]}], lr=0.1,
                  momentum=0.9, nesterov=True)
    ob = torch.optim.SGD([{"params": b[:1], "weight_decay": 1e-3}, {"params": b[1:]}], lr=0.1,
                         momentum=0.9, nesterov=True)
    for _ in range(3):
        grads = [torch.randn(5, 3, generator=g) for _ in range(2)]
        for ps in (a, b):
            for p, gr in zip(ps, grads):
                p.grad = gr.clone()
        oa.step()
        ob.step()
    for p, q in zip(a, b):
        assert torch.equal(p, q)


def test_fused_sgd_fallback_returns_the_closure_loss():
    """torch.optim.SGD.step(closure) returns the closure's loss; so must the fallback path
    (the closure is evaluated once, before the stock update)."""
    from shiftgcn.train import FusedSGD
    p = torch.nn.Parameter(torch.ones(4))
    opt = FusedSGD([p], lr=0.1, momentum=0.9)
    calls = []

    def closure():
        calls.append(1)
        opt.zero_grad()
        loss = (p * p).sum()
        loss.backward()
        return loss

    loss = opt.step(closure)
    assert loss is not None and float(loss) == 4.0
    assert len(calls) == 1
    assert torch.allclose(p.detach(), torch.full((4,), 0.8))


def test_param_groups_track_hyper_parameter_assignments():
    """Round 6: FusedSGD's parameter groups write every lr / weight_decay assignment into the
    device pairs a graph-captured step reads (here a CPU stand-in for the device table), also
    after load_state_dict / add_param_group, through an LR scheduler, and survive deepcopy,
    pickling and a state_dict round trip with the stock optimizer."""
    import copy
    import io
    from shiftgcn.train import FusedSGD, _HyperGroup, adjust_learning_rate
    ps = [torch.nn.Parameter(torch.ones(3)) for _ in range(3)]
    opt = FusedSGD([{"params": ps[:1], "weight_decay": 1e-3}, {"params": ps[1:2]}], lr=0.1,
                   momentum=0.9, nesterov=True)
    assert all(isinstance(g, _HyperGroup) for g in opt.param_groups)
    opt._hyper = torch.zeros(2, 2)                  # what the first eager CUDA step makes
    opt._hyper_host = [None, None]
    for g in opt.param_groups:
        opt._hyper_changed(g)
    assert opt._hyper.tolist() == [[torch.tensor(1e-3).item(), torch.tensor(0.1).item()],
                                   [0.0, torch.tensor(0.1).item()]]
    adjust_learning_rate(opt, 60)                    # main.py:342-353: x0.1 at epoch 60
    assert opt._hyper[:, 1].tolist() == [torch.tensor(0.01).item()] * 2
    sched = torch.optim.lr_scheduler.StepLR(opt, step_size=1, gamma=0.5)
    for p in ps:
        p.grad = torch.zeros(3)
    opt.step()
    sched.step()
    assert opt._hyper[:, 1].tolist() == [torch.tensor(0.005).item()] * 2
    sd = opt.state_dict()
    opt.load_state_dict(sd)                          # new group dicts: wrapped again
    assert all(isinstance(g, _HyperGroup) for g in opt.param_groups)
    opt.param_groups[1]["lr"] = 0.25
    assert opt._hyper[1, 1].item() == 0.25
    opt.add_param_group({"params": ps[2:]})         # the device table is re-made (3 groups)
    assert opt._hyper is None and isinstance(opt.param_groups[2], _HyperGroup)
    stock = torch.optim.SGD(ps, lr=0.1, momentum=0.9)
    stock_sd = copy.deepcopy(opt.state_dict())
    assert stock_sd["param_groups"][1]["lr"] == 0.25 and type(stock_sd["param_groups"][1]) is dict
    torch.optim.SGD([{"params": ps[:1]}, {"params": ps[1:2]}, {"params": ps[2:]}],
                    lr=0.1).load_state_dict(stock_sd)
    del stock
    twin = copy.deepcopy(opt)
    assert twin.param_groups[0]._opt is twin
    buf = io.BytesIO()
    torch.save(opt, buf)
    assert buf.tell() > 0
