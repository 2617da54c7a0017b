"""Write a synthetic dataset in the reference's on-disk format (feeders/feeder.py:41-60,
data_gen/ntu_gendata.py:137-139): (N, 3, T, V, M) float32 .npy + (sample_name, label)
pickle, for `bench.py --data/--labels` runs.
    python tools/make_clip_dataset.py OUTDIR [--n 256] [--config ntu|mp]"""
import argparse
import os
import pickle

import numpy as np

SHAPES = {"ntu": (300, 25, 2, 60), "mp": (300, 33, 1, 2)}

ap = argparse.ArgumentParser()
ap.add_argument("out")
ap.add_argument("--n", type=int, default=256)
ap.add_argument("--config", default="ntu", choices=sorted(SHAPES))
a = ap.parse_args()
T, V, M, K = SHAPES[a.config]
os.makedirs(a.out, exist_ok=True)
rng = np.random.default_rng(0)
data = np.lib.format.open_memmap(os.path.join(a.out, "data.npy"), mode="w+",
                                 dtype=np.float32, shape=(a.n, 3, T, V, M))
for i in range(0, a.n, 64):
    data[i:i + 64] = rng.standard_normal(data[i:i + 64].shape, dtype=np.float32)
data.flush()
with open(os.path.join(a.out, "label.pkl"), "wb") as f:
    pickle.dump(([f"clip{i:06d}" for i in range(a.n)],
                 [int(v) for v in rng.integers(0, K, a.n)]), f)
print(os.path.join(a.out, "data.npy"), os.path.join(a.out, "label.pkl"))
