"""Debug: the chain test with the side finalizes batched (SGCN_BATCH_SIDE) on and off."""
import os
import sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "..", "shift-gcn_amd"),
                os.path.join(os.path.dirname(__file__), "..", "..", "tests", "golden"),
                os.path.join(os.path.dirname(__file__), "..", "..")]
import torch
import formula
import shiftgcn
from shiftgcn import fused
from shiftgcn.shift_gcn import linked_units

res = {}
for batch in (0, 1):
    fused.BATCH_SIDE = batch
    torch.manual_seed(0)
    ours = torch.nn.Sequential(shiftgcn.TCN_GCN_unit(64, 64, None, num_point=25),
                               shiftgcn.TCN_GCN_unit(64, 128, None, residual=False,
                                                     num_point=25))
    formula.fill_state(ours, seed=41)
    ours = ours.cuda().train()
    x = formula.tensor((3, 64, 16, 25), 42, 1.0).cuda().requires_grad_(True)
    g = formula.tensor((3, 128, 16, 25), 43, 1.0).cuda()
    with linked_units(list(ours)):
        y = ours(x)
    y.backward(g)
    torch.cuda.synchronize()
    res[batch] = {n: p.grad.clone() for n, p in ours.named_parameters() if p.grad is not None}
    print("batch", batch, "deferred left:", {k: (len(v.pos), len(v.mask)) for k, v in fused._TASKS.items()})
for n in res[0]:
    d = (res[0][n] - res[1][n]).abs().max().item()
    if d > 0:
        print("DIFF", n, d, res[0][n].abs().max().item(), res[1][n].abs().max().item())
print("done")

# ops level: the batched finalizes vs one launch each
from shiftgcn import ops
g = torch.Generator().manual_seed(1)
ents, ref = [], []
for C in (8, 64, 3):
    B = 5
    ws = torch.randn(B * C * 2, generator=g).cuda()
    pp = ops.PosPartials(ws, B, C)
    gx, gy = torch.full((C,), 7.0, device="cuda"), torch.full((C,), 7.0, device="cuda")
    rx, ry = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
    pp.finalize(rx, ry)
    ents.append((pp, gx, gy))
    ref.append((rx, ry))
ops.pos_finalize_many(ents)
torch.cuda.synchronize()
for (pp, gx, gy), (rx, ry) in zip(ents, ref):
    print("pos many ok:", torch.equal(gx, rx), torch.equal(gy, ry))
masks = [torch.randn(1, 25, c, generator=g).cuda() for c in (3, 64, 128)]
outs = ops.mask_prep_many(masks)
print("mask prep many ok:", all(torch.equal(o, ops.mask_prep(m)) for o, m in zip(outs, masks)))
mg = []
for m in masks:
    C, V, B = m.shape[2], 25, 4
    part = torch.randn(B * C * V, generator=g).cuda()
    d1, d2 = torch.empty_like(m), torch.empty_like(m)
    ops.mask_grad_finalize(part, m, B, C, V, out=d1)
    mg.append((part, m, B, C, V, d2, d1))
ops.mask_grad_finalize_many([e[:6] for e in mg])
torch.cuda.synchronize()
print("mask grad many ok:", all(torch.equal(e[5], e[6]) for e in mg))
