"""Isolated timing of the shift_in backward variants at one NTU unit shape (B=128, C=64,
T=300, V=25): plain (affine + BN partials) vs GBN (+ Shift_gcn.bn's per-joint sums).
    python tools/bench/gbn_probe.py [C T]"""
import sys

import torch

sys.path.insert(0, "shift-gcn_amd")
from shiftgcn import ops  # noqa: E402

C = int(sys.argv[1]) if len(sys.argv) > 1 else 64
T = int(sys.argv[2]) if len(sys.argv) > 2 else 300
B, V = 128, 25
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
gout = torch.randn(B, C, T, V, device=dev, generator=g)
H = torch.relu(torch.randn(B, C, T, V, device=dev, generator=g))
Z = torch.randn(B, C, T, V, device=dev, generator=g)
xpos = torch.empty(C, device=dev).uniform_(-1e-8, 1e-8)
ypos = torch.empty(C, device=dev).uniform_(-1, 1)
st = ops.BnStats(C, dev)
for t in (st.mean, st.invstd, st.scale, st.shift):
    t.copy_(torch.rand(C, device=dev) + 0.5)
zst = ops.BnStats(C * V, dev)
for t in (zst.mean, zst.invstd, zst.scale, zst.shift):
    t.copy_(torch.rand(C * V, device=dev) + 0.5)


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


T1 = 4 * B * C * T * V
plain = timeit(lambda: ops.tshift_bwd(gout, H, xpos, ypos, 1, scale=st.scale, shift=st.shift,
                                      bn_stats=st))
gbn = timeit(lambda: ops.tshift_bwd_gbn(gout, H, xpos, ypos, st, Z, zst))
bnin = timeit(lambda: ops.tshift_bwd_bnin(gout, H, Z, torch.ones(3, C, device=dev), H, xpos,
                                          ypos))
noaff = timeit(lambda: ops.tshift_bwd(gout, H, xpos, ypos, 1))
relu = timeit(lambda: ops.tshift_bwd(gout, H, xpos, ypos, 1, relu_mask=True))
aff = timeit(lambda: ops.tshift_bwd(gout, H, xpos, ypos, 1, scale=st.scale, shift=st.shift))
print(f"C={C} T={T}: bare {noaff:.1f} us | relu {relu:.1f} | affine {aff:.1f} | "
      f"affine+BNP {plain:.1f}")
print(f"C={C} T={T}: plain(affine+BNP) {plain:.1f} us ({3 * T1 / plain / 1e6:.2f} TB/s) | "
      f"GBN {gbn:.1f} us ({4 * T1 / gbn / 1e6:.2f} TB/s) | bnin {bnin:.1f} us "
      f"({5 * T1 / bnin / 1e6:.2f} TB/s)")
