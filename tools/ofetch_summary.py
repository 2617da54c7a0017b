"""Summarise tools/gpu_ofetch.sh (rocprofv3 PMC passes over tools/bench/ofetch builds):
per build variant and unit shape, the forward contraction's HBM-side counters averaged over
the 5 timed launches (the warm-up launch dropped), next to the algorithmic bytes.

    python tools/ofetch_summary.py gpurun_out/r04b/ofetch
"""
import csv
import os
import re
import sys
from collections import defaultdict

SHAPES = ["l2 gcn 64<-64 T300", "l5 gcn 128<-64 T300", "l5 down 128<-64 T300",
          "l6 tcn 128<-128 T150", "l8 gcn 256<-128 T150", "l8 down 256<-128 T150",
          "l9 tcn 256<-256 T75", "l8 dX acc 128<-256 T150"]
PER_SHAPE = 6   # 1 warm-up + 5 timed launches


def passes(vdir):
    out = defaultdict(dict)   # counter -> {dispatch index: value}
    for p in sorted(os.listdir(vdir)):
        f = os.path.join(vdir, p, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        rows = [r for r in csv.DictReader(open(f)) if "pwg_fwd_kernel" in r["Kernel_Name"]
                or "pw_fwd_smallm" in r["Kernel_Name"]]
        ids = sorted({int(r["Dispatch_Id"]) for r in rows})
        pos = {d: i for i, d in enumerate(ids)}
        for r in rows:
            out[r["Counter_Name"]][pos[int(r["Dispatch_Id"])]] = float(r["Counter_Value"])
    return out


def times(path):
    t = {}
    if os.path.exists(path):
        for line in open(path):
            m = re.match(r"(.+?)\s+([\d.]+) us", line)
            if m:
                t[m.group(1).strip()] = float(m.group(2))
    return t


def main(root):
    variants = [v for v in ("prod", "noxcd", "d1", "d2", "xnt", "asc1") if os.path.isdir(os.path.join(root, v))]
    print(f"{'shape':26s} {'var':5s} {'us':>7s} {'FETCHx2 MB':>10s} {'WRITE MB':>9s} "
          f"{'L2 hit':>7s} {'RDREQ M':>8s} {'RD32B M':>8s}")
    for si, shape in enumerate(SHAPES):
        for v in variants:
            c = passes(os.path.join(root, v))
            tt = times(os.path.join(root, f"time_{v}.txt"))

            def avg(name):
                d = c.get(name, {})
                vals = [d[i] for i in range(si * PER_SHAPE + 1, (si + 1) * PER_SHAPE) if i in d]
                return sum(vals) / len(vals) if vals else float("nan")
            fetch = 2 * avg("FETCH_SIZE") * 1024 / 1e6
            write = avg("WRITE_SIZE") * 1024 / 1e6
            hit, miss = avg("TCC_HIT_sum"), avg("TCC_MISS_sum")
            hr = hit / (hit + miss) if hit + miss > 0 else float("nan")
            print(f"{shape:26s} {v:5s} {tt.get(shape, float('nan')):7.1f} {fetch:10.1f} "
                  f"{write:9.1f} {hr:7.3f} {avg('TCC_EA0_RDREQ_sum') / 1e6:8.3f} "
                  f"{avg('TCC_EA0_RDREQ_32B_sum') / 1e6:8.3f}")
        print()


if __name__ == "__main__":
    main(sys.argv[1])
