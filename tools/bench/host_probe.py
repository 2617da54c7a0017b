"""Host-side cost of one NTU training step (tuning harness): the enqueue time per step with
the GPU left running (no sync inside the loop) against the GPU time per step, and a
cProfile of the host's top functions over a few steps.
    python tools/bench/host_probe.py [--steps 10]"""
import cProfile
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "shift-gcn_amd"))
import torch  # noqa: E402

import shiftgcn  # noqa: E402
from shiftgcn import train  # noqa: E402

steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 10
torch.manual_seed(0)
model = shiftgcn.Model(num_class=60, num_point=25, num_person=2,
                       graph="graph.ntu_rgb_d.Graph").cuda().train()
opt = train.build_optimizer(model, base_lr=0.1)
x = torch.randn(64, 3, 300, 25, 2, device="cuda")
y = torch.randint(0, 60, (64,), device="cuda")
for _ in range(5):
    train.train_step(model, opt, x, y)
torch.cuda.synchronize()
# host enqueue time per step while the GPU runs behind (a deep queue: host far ahead?)
ts = []
t_start = time.perf_counter()
for _ in range(steps):
    t0 = time.perf_counter()
    train.train_step(model, opt, x, y)
    ts.append(time.perf_counter() - t0)
t_enq = time.perf_counter() - t_start
torch.cuda.synchronize()
t_all = time.perf_counter() - t_start
print(f"host enqueue per step: {1e3 * sum(ts) / steps:.2f} ms (min {1e3 * min(ts):.2f}, "
      f"max {1e3 * max(ts):.2f}); wall per step incl. drain {1e3 * t_all / steps:.2f} ms; "
      f"enqueue total {1e3 * t_enq:.1f} ms")
print("per step ms:", " ".join(f"{1e3 * t:.1f}" for t in ts))
pr = cProfile.Profile()
pr.enable()
for _ in range(steps):
    train.train_step(model, opt, x, y)
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(25)
