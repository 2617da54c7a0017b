"""Debug: fused gcn dX (SGCN_GCN_DX_FUSED) vs the two-launch form, per parameter."""
import sys
sys.path.insert(0, "tests/golden")
sys.path.insert(0, "shift-gcn_amd")
import torch
import formula
import shiftgcn
from shiftgcn import fused
from shiftgcn.shift_gcn import linked_units

DEV = "cuda"


def run(flag, mk, x, gy, link):
    fused.GCN_DX_FUSED = flag
    m = mk()
    xo = x.clone().requires_grad_(True)
    if link:
        with linked_units(list(m)):
            y = m(xo)
    else:
        y = m(xo)
    y.backward(gy)
    torch.cuda.synchronize()
    g = {n: p.grad.double().cpu() for n, p in m.named_parameters() if p.grad is not None}
    g["x"] = xo.grad.double().cpu()
    return g


def cmp(name, mk, x, gy, link):
    a, b = run(1, mk, x, gy, link), run(0, mk, x, gy, link)
    worst = sorted(((float((a[k] - b[k]).abs().max()) / max(float(b[k].abs().max()), 1e-30), k)
                    for k in b), reverse=True)[:6]
    print(name, [(k, f"{e:.2e}") for e, k in worst])


def unit(cin, cout, res=True, stride=1):
    def mk():
        u = shiftgcn.TCN_GCN_unit(cin, cout, None, stride=stride, residual=res, num_point=25)
        formula.fill_state(u, seed=3)
        return torch.nn.Sequential(u).to(DEV).train()
    return mk


def chain():
    def mk():
        s = torch.nn.Sequential(shiftgcn.TCN_GCN_unit(64, 64, None, num_point=25),
                                shiftgcn.TCN_GCN_unit(64, 64, None, num_point=25),
                                shiftgcn.TCN_GCN_unit(64, 64, None, num_point=25))
        formula.fill_state(s, seed=4)
        return s.to(DEV).train()
    return mk


x = formula.tensor((3, 64, 16, 25), 1, 1.0).to(DEV)
gy = formula.tensor((3, 64, 16, 25), 2, 1.0).to(DEV)
cmp("unit64", unit(64, 64), x, gy, False)
cmp("chain3 linked", chain(), x, gy, True)
cmp("chain3 unlinked", chain(), x, gy, False)
gy2 = formula.tensor((3, 128, 8, 25), 2, 1.0).to(DEV)
cmp("unit64-128 s2", unit(64, 128, True, 2), x, gy2, False)
fused.ASYNC_DW = 0
cmp("chain3 linked, no side stream", chain(), x, gy, True)
fused.ASYNC_DW = 1
fused.TAIL_MAIN = 0
cmp("chain3 linked, TAIL_MAIN 0", chain(), x, gy, True)
fused.TAIL_MAIN = 3
a, b = run(1, chain(), x, gy, True), run(0, chain(), x, gy, True)
print("fused", a["0.gcn1.Linear_bias"].flatten()[:6].tolist())
print("2-launch", b["0.gcn1.Linear_bias"].flatten()[:6].tolist())
