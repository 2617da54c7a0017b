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
