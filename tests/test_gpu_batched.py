"""Optimizer-only finalizes batched into one launch per kind (round 4, `fused.BATCH_SIDE`):
`sgcn_tshift_pos_finalize_many`, `sgcn_mask_prep_many`, `sgcn_mask_grad_finalize_many`
must write exactly what their one-launch-per-entry forms write (the position gradients of
`shift_cuda_kernel.cu:501-509` + `shift.py:20-30`, tanh(Feature_Mask) + 1 of
`shift_gcn.py:134`, the mask gradient), for mixed shapes and for more entries than one
launch takes (`SGCN_BATCH_MAX`: the wrappers chunk), and a linked chain's gradients must be
bit-identical with the batching on and off."""
import pytest
import torch

import formula

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _gen(seed):
    return torch.Generator().manual_seed(seed)


@pytest.mark.parametrize("n", [1, 3, 33, 70])
def test_pos_finalize_many_bit_identical(n):
    from shiftgcn import ops
    g = _gen(n)
    shapes = [(5, 8), (3, 64), (2, 3), (7, 128), (1, 256)]
    ents, ref = [], []
    for k in range(n):
        B, C = shapes[k % len(shapes)]
        ws = torch.randn(B * C * 2, generator=g).to(DEV)
        pp = ops.PosPartials(ws, B, C)
        rx, ry = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
        pp.finalize(rx, ry)
        ox, oy = torch.full((C,), 7.0, device=DEV), torch.full((C,), 7.0, device=DEV)
        ents.append((pp, ox, oy))
        ref.append((rx, ry))
    ops.pos_finalize_many(ents)
    torch.cuda.synchronize()
    for (_, ox, oy), (rx, ry) in zip(ents, ref):
        assert torch.equal(ox, rx) and torch.equal(oy, ry)


@pytest.mark.parametrize("n", [1, 10, 40])
def test_mask_prep_many_bit_identical(n):
    from shiftgcn import ops
    g = _gen(100 + n)
    masks = [torch.randn(1, 25, (3, 64, 128, 256)[k % 4], generator=g).to(DEV)
             for k in range(n)]
    outs = ops.mask_prep_many(masks)
    torch.cuda.synchronize()
    assert len(outs) == n
    for o, m in zip(outs, masks):
        assert torch.equal(o, ops.mask_prep(m))
        assert torch.allclose(o, torch.tanh(m) + 1, atol=1e-6, rtol=0)


@pytest.mark.parametrize("n", [1, 5, 35])
def test_mask_grad_finalize_many_bit_identical(n):
    from shiftgcn import ops
    g = _gen(200 + n)
    ents, ref = [], []
    for k in range(n):
        C, V, B = (3, 64, 128, 256)[k % 4], (25, 33)[k % 2], (4, 2, 6)[k % 3]
        m = torch.randn(1, V, C, generator=g).to(DEV)
        part = torch.randn(B * C * V, generator=g).to(DEV)
        want, got = torch.empty_like(m), torch.full_like(m, 5.0)
        ops.mask_grad_finalize(part, m, B, C, V, out=want)
        ents.append((part, m, B, C, V, got))
        ref.append(want)
    ops.mask_grad_finalize_many(ents)
    torch.cuda.synchronize()
    for e, want in zip(ents, ref):
        assert torch.equal(e[5], want)


def test_linked_chain_batching_bit_identical(monkeypatch):
    import shiftgcn
    from shiftgcn import fused
    from shiftgcn.shift_gcn import linked_units
    res = {}
    for batch in (0, 1):
        monkeypatch.setattr(fused, "BATCH_SIDE", batch)
        torch.manual_seed(0)
        ours = torch.nn.Sequential(
            shiftgcn.TCN_GCN_unit(64, 64, None, num_point=25),
            shiftgcn.TCN_GCN_unit(64, 64, None, num_point=25),
            shiftgcn.TCN_GCN_unit(64, 128, None, residual=False, num_point=25))
        formula.fill_state(ours, seed=41)
        ours = ours.to(DEV).train()
        x = formula.tensor((3, 64, 16, 25), 42, 1.0).to(DEV).requires_grad_(True)
        gy = formula.tensor((3, 128, 16, 25), 43, 1.0).to(DEV)
        with linked_units(list(ours)):
            y = ours(x)
        y.backward(gy)
        torch.cuda.synchronize()
        assert not fused._TASKS   # every backward's deferred work was flushed
        res[batch] = ({n: p.grad.clone() for n, p in ours.named_parameters()
                       if p.grad is not None}, x.grad.clone())
    (g0, x0), (g1, x1) = res[0], res[1]
    assert g0.keys() == g1.keys() and len(g0) > 20
    for n in g0:
        assert torch.equal(g0[n], g1[n]), n
    assert torch.equal(x0, x1)
