"""Debug: EnsembleGraph recaptures and per-batch time (round-6 ENS check)."""
import sys
import time
sys.path.insert(0, "shift-gcn_amd")
import torch
import shiftgcn
from shiftgcn import ensemble as E

dev = torch.device("cuda:0")
torch.manual_seed(1)
models = [shiftgcn.Model(num_class=2, num_point=33, num_person=1,
                         graph="graph.mediapipe_pose.Graph").to(dev).eval() for _ in range(4)]
ens = E.Ensemble(models).to(dev)
x = torch.randn(256, 3, 300, 33, 1, device=dev)
g = E.EnsembleGraph(ens, x.shape, dev)
for _ in range(5):
    g.run(x)
torch.cuda.synchronize()
print("captures after warm-up", g.captures, "epoch", E._MODULE_EPOCH[0])
t0 = time.perf_counter()
for _ in range(20):
    g.run(x)
torch.cuda.synchronize()
print("ms per batch", (time.perf_counter() - t0) / 20 * 1e3, "captures", g.captures)
# host cost of the state key
t0 = time.perf_counter()
for _ in range(100):
    E._state_key(g._mods)
print("state key ms", (time.perf_counter() - t0) / 100 * 1e3)
# without the key check at all: replay only
t0 = time.perf_counter()
for _ in range(20):
    g.static_in.copy_(x, non_blocking=True)
    g.graph.replay()
torch.cuda.synchronize()
print("replay-only ms per batch", (time.perf_counter() - t0) / 20 * 1e3)
