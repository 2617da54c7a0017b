"""Per-launch cost of the producer-tail BatchNorm finalize (sgcn_moments_fin) against
sgcn_moments + sgcn_bn_finalize at the NTU unit shapes (tuning probe, not a test)."""
import os
import sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "..", "shift-gcn_amd")]
import torch

from shiftgcn import ops

DEV = "cuda"


def timeit(fn, n=50):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / n


for (B, C, T, V) in [(128, 64, 300, 25), (128, 128, 150, 25), (128, 256, 75, 25),
                     (128, 128, 300, 25)]:
    x = torch.randn(B, C, T, V, device=DEV)
    for pj in (3, 0):
        F = C * (V if pj else 1)
        n_part = T if pj else T * V
        bn = (torch.nn.BatchNorm1d(F) if pj else torch.nn.BatchNorm2d(C)).to(DEV)
        part = ops.moments(x, pj)
        t_m = timeit(lambda: ops.moments(x, pj))
        t_f = timeit(lambda: ops.bn_finalize(part, B, F, n_part, bn, perm_V=V if pj else 0))
        t_mf = timeit(lambda: ops.bn_finalize(ops.moments(x, pj), B, F, n_part, bn,
                                              perm_V=V if pj else 0))
        t_t = timeit(lambda: ops.moments_bn(x, pj, bn))
        print(f"B{B} C{C} T{T} V{V} pj{pj}: moments {t_m:7.1f} us  finalize {t_f:6.1f}  "
              f"both {t_mf:7.1f}  tail {t_t:7.1f}  (tail - both {t_t - t_mf:+6.1f})", flush=True)
