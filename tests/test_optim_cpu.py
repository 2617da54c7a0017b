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
