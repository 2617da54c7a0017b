"""Per-launch-shape time table of the NTU training step (HIP events around every C-ABI
launch, keyed by op + shape): which contraction / streaming pass costs what, and at what
fraction of its own roofline (FP32 MFMA 157.3 TF or HBM 8 TB/s, algorithmic work).
    python tools/shape_breakdown.py [--steps 3] [--batch 64] [--config ntu|mp]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (os.path.join(REPO, "shift-gcn_amd"), REPO):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402

import shiftgcn  # noqa: E402
from shiftgcn import ops, train  # noqa: E402

CFG = {"ntu": (60, 25, 2, "graph.ntu_rgb_d.Graph"), "mp": (2, 33, 1, "graph.mediapipe_pose.Graph")}

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=3)
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--config", default="ntu", choices=sorted(CFG))
a = ap.parse_args()
K, V, M, graph = CFG[a.config]
torch.manual_seed(1)
model = shiftgcn.Model(num_class=K, num_point=V, num_person=M, graph=graph).cuda().train()
opt = train.build_optimizer(model, base_lr=0.1)
g = torch.Generator().manual_seed(0)
x = torch.randn(a.batch, 3, 300, V, M, generator=g).cuda()
y = torch.randint(0, K, (a.batch,), generator=g).cuda()
for _ in range(3):
    train.train_step(model, opt, x, y)
torch.cuda.synchronize()
timer = ops.LaunchTimer(detail=True)
ops.set_launch_timer(timer)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(a.steps):
    train.train_step(model, opt, x, y)
e1.record()
torch.cuda.synchronize()
ops.set_launch_timer(None)
step_ms = e0.elapsed_time(e1) / a.steps
summ = timer.summary()
rows = sorted(summ.items(), key=lambda kv: -kv[1]["ms_total"])
tot = sum(v["ms_total"] for v in summ.values()) / a.steps
print(f"step {step_ms:.3f} ms (event-timed), launches timed {tot:.3f} ms")
print(f"{'ms/step':>8} {'n':>3} {'us/launch':>9} {'TF/s':>7} {'TB/s':>6} {'roof':>5}  op")
for k, v in rows:
    n = v["launches"] // a.steps
    ms = v["ms_total"] / a.steps
    s = v["ms_total"] / 1e3
    tf = v["flops"] / s / 1e12 if s else 0
    tb = v["bytes"] / s / 1e12 if s else 0
    print(f"{ms:8.3f} {n:3d} {1e3 * ms / max(n, 1):9.1f} {tf:7.1f} {tb:6.2f} "
          f"{v['roof_ms'] / v['ms_total']:5.2f}  {k}")
