"""Native model head and tail (reference model/shift_gcn.py:193-216).

* ``head.data_bn_planes`` == permute -> ``nn.BatchNorm1d(M*V*C)`` -> permute back, against a
  plain PyTorch fp32 copy of the same module: output, running statistics and
  num_batches_tracked, data_bn's weight/bias gradients and the clip gradient, in train and
  eval mode, for V*M above one 256-thread column tile, ragged T, M = 1;
* ``head.pool`` == ``x.view(N, M, C, -1).mean(3).mean(1)``; its backward bit for bit
  (same division order as autograd's mean backward);
* the error behaviour of ``F.batch_norm`` (one value per channel in training).
Tolerance: 1e-5 relative to the tensor's max magnitude (north_star's fp32 bar).
"""
import copy

import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu
DEV = "cuda"

CASES = [
    # (N, C, T, V, M)
    (4, 3, 300, 25, 2),        # NTU clip shape
    (3, 3, 17, 33, 1),         # MP body: V=33, one person, ragged T
    (2, 3, 9, 25, 12),         # V*M = 300 > 256: two column tiles
    (1, 2, 5, 7, 3),
]


def _ref_head(bn, x):
    N, C, T, V, M = x.shape
    y = x.permute(0, 4, 3, 1, 2).contiguous().view(N, M * V * C, T)
    y = bn(y)
    return y.view(N, M, V, C, T).permute(0, 1, 3, 4, 2).contiguous().view(N * M, C, T, V)


def _close(a, b, what, tol=1e-5):
    a, b = a.detach().double(), b.detach().double()
    err = float((a - b).abs().max())
    scale = float(b.abs().max()) + 1e-30
    assert err <= tol * scale + 1e-7, (what, err, scale)


@pytest.mark.parametrize("training", [True, False], ids=["train", "eval"])
@pytest.mark.parametrize("case", CASES, ids=["x".join(map(str, c)) for c in CASES])
def test_data_bn_planes_matches_torch(case, training):
    from shiftgcn import head
    N, C, T, V, M = case
    g = torch.Generator().manual_seed(sum(case) + training)
    F = M * V * C
    bn_ref = nn.BatchNorm1d(F)
    with torch.no_grad():
        bn_ref.weight.copy_(torch.rand(F, generator=g) + 0.5)
        bn_ref.bias.copy_(torch.randn(F, generator=g))
        bn_ref.running_mean.copy_(torch.randn(F, generator=g))
        bn_ref.running_var.copy_(torch.rand(F, generator=g) + 0.5)
    bn_ref = bn_ref.to(DEV).train(training)
    bn = copy.deepcopy(bn_ref)
    x = (torch.randn(N, C, T, V, M, generator=g) * 3 + 1).to(DEV)
    gy = torch.randn(N * M, C, T, V, generator=g).to(DEV)
    xr = x.clone().requires_grad_(True)
    yr = _ref_head(bn_ref, xr)
    yr.backward(gy)
    xo = x.clone().requires_grad_(True)
    yo = head.data_bn_planes(bn, xo)
    yo.backward(gy)
    torch.cuda.synchronize()
    assert yo.shape == (N * M, C, T, V)
    _close(yo, yr, "y")
    _close(bn.running_mean, bn_ref.running_mean, "running_mean")
    _close(bn.running_var, bn_ref.running_var, "running_var")
    assert int(bn.num_batches_tracked) == int(bn_ref.num_batches_tracked)
    _close(bn.weight.grad, bn_ref.weight.grad, "dgamma")
    _close(bn.bias.grad, bn_ref.bias.grad, "dbeta")
    _close(xo.grad, xr.grad, "dx")


def test_data_bn_planes_skips_clip_gradient_when_not_required():
    from shiftgcn import head, ops
    N, C, T, V, M = 2, 3, 20, 25, 2
    bn = nn.BatchNorm1d(M * V * C).to(DEV).train()
    x = torch.randn(N, C, T, V, M, device=DEV)
    calls = []
    real = ops.head_bwd_apply
    try:
        ops.head_bwd_apply = lambda *a: calls.append(1) or real(*a)
        head.data_bn_planes(bn, x).sum().backward()
    finally:
        ops.head_bwd_apply = real
    torch.cuda.synchronize()
    assert calls == [] and bn.weight.grad is not None


def test_data_bn_planes_one_value_per_channel_raises():
    from shiftgcn import head
    bn = nn.BatchNorm1d(2 * 25 * 3).to(DEV).train()
    with pytest.raises(ValueError, match="Expected more than 1 value per channel"):
        head.data_bn_planes(bn, torch.randn(1, 3, 1, 25, 2, device=DEV))
    bn.eval()   # eval mode: running statistics, any batch size
    head.data_bn_planes(bn, torch.randn(1, 3, 1, 25, 2, device=DEV))


def test_data_bn_planes_rejects_cpu_input():
    from shiftgcn import head
    bn = nn.BatchNorm1d(150)
    with pytest.raises(RuntimeError, match="must be a CUDA tensor"):
        head.data_bn_planes(bn, torch.randn(2, 3, 4, 25, 2))


@pytest.mark.parametrize("shape", [(4, 2, 256, 75, 25), (3, 1, 64, 9, 33), (2, 3, 5, 1, 1)])
def test_pool_matches_torch(shape):
    from shiftgcn import head
    N, M, C, T, V = shape
    g = torch.Generator().manual_seed(N * 7 + C)
    x = torch.randn(N * M, C, T, V, generator=g).to(DEV)
    dout = torch.randn(N, C, generator=g).to(DEV)
    xr = x.clone().requires_grad_(True)
    pr = xr.view(N, M, C, -1).mean(3).mean(1)
    pr.backward(dout)
    xo = x.clone().requires_grad_(True)
    po = head.pool(xo, N, M)
    po.backward(dout)
    torch.cuda.synchronize()
    _close(po, pr, "pool")
    assert torch.equal(xo.grad, xr.grad)       # same divisions, same order


def test_model_uses_native_head(monkeypatch):
    """Model.forward runs data_bn and the pooling through the HIP head (no torch BN)."""
    import shiftgcn
    from shiftgcn import ops
    seen = []
    for name in ("head_moments", "head_apply", "pool", "head_bwd_reduce", "pool_bwd"):
        real = getattr(ops, name)
        monkeypatch.setattr(ops, name, (lambda r, n: lambda *a, **k: seen.append(n) or r(*a, **k))(
            real, name))

    def no_torch_bn(*a, **k):
        raise AssertionError("torch batch_norm called")

    m = shiftgcn.Model(num_class=60, num_point=25, num_person=2,
                       graph="graph.ntu_rgb_d.Graph").to(DEV).train()
    monkeypatch.setattr(m.data_bn, "forward", no_torch_bn)
    x = torch.randn(2, 3, 16, 25, 2, device=DEV)
    m(x).sum().backward()
    torch.cuda.synchronize()
    assert sorted(set(seen)) == sorted(["head_moments", "head_apply", "pool", "head_bwd_reduce",
                                        "pool_bwd"]), seen
    assert m.data_bn.weight.grad is not None and int(m.data_bn.num_batches_tracked) == 1
