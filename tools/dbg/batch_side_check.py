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
    print("batch", batch, "deferred left:", {k: (len(v["pos"]), len(v["mask"])) for k, v in fused._DEFER.items()})
for n in res[0]:
    d = (res[0][n] - res[1][n]).abs().max().item()
    if d > 0:
        print("DIFF", n, d, res[0][n].abs().max().item(), res[1][n].abs().max().item())
print("done")
