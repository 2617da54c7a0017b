"""Per-kernel HBM traffic from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

    python tools/pmc_summary.py <pmc_dir> [--match SUBSTR] [--last N]

FETCH_SIZE / WRITE_SIZE are reported in KB per dispatch. gfx950 correction
(MI355X_MICROARCH.md §HBM): FETCH_SIZE counts 64 B per 128-B request of a wide
coalesced read, so it is DOUBLED here ("fetch_corr"); WRITE_SIZE is taken as is.
Dispatches are keyed by (kernel, grid) and averaged over the run.
"""
import argparse
import csv
import os
from collections import OrderedDict


def read(path, counter):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            out.append((r["Kernel_Name"], r["Grid_Size"], float(r["Counter_Value"]) * 1024.0,
                        int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    return out


def short(n):
    n = n.replace("sgcn::(anonymous namespace)::", "")
    if n.startswith("void "):
        n = n[5:]
    i = n.find("(")
    return n[:i] if i > 0 else n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    f = read(os.path.join(a.dir, "FETCH_SIZE", "run_counter_collection.csv"), "FETCH_SIZE")
    w = read(os.path.join(a.dir, "WRITE_SIZE", "run_counter_collection.csv"), "WRITE_SIZE")
    agg = OrderedDict()
    for (n, g, fb, _), (n2, g2, wb, _) in zip(f, w):
        if n != n2 or a.match not in n:
            continue
        d = agg.setdefault((short(n), g), [0, 0.0, 0.0])
        d[0] += 1
        d[1] += fb
        d[2] += wb
    print(f"{'kernel':70s} {'grid':>9s} {'n':>4s} {'fetchx2 MB':>11s} {'write MB':>9s}")
    for (n, g), (c, fb, wb) in agg.items():
        print(f"{n[:70]:70s} {g:>9s} {c:4d} {2 * fb / c / 1e6:11.1f} {wb / c / 1e6:9.1f}")


if __name__ == "__main__":
    main()
