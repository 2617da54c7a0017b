"""Summarise a rocprofv3 kernel trace (rocpd .db or kernel_trace.csv).

    python tools/kernel_stats.py <results.db|kernel_trace.csv> [--steps K] [--csv out.csv]
        [--timeline]

Prints per-kernel totals (the `--stats` view) and, with --timeline, the dispatch sequence
of the LAST training step (steps are delimited by the optimizer's first kernel), with each
dispatch's duration — the per-launch view used to price fusions in DESIGN.md.
"""
import argparse
import csv
import sqlite3
import sys
from collections import OrderedDict


def load(path):
    rows = []
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, start, end, gx, gy, gz, wx in c.execute(
                "select name, start, end, grid_x, grid_y, grid_z, workgroup_x from kernels "
                "order by start"):
            rows.append((name, int(start), int(end), (gx, gy, gz, wx)))
    else:
        with open(path) as f:
            for r in csv.DictReader(f):
                rows.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                             (r.get("Grid_Size_X"), r.get("Grid_Size_Y"), r.get("Grid_Size_Z"),
                              r.get("Workgroup_Size_X"))))
        rows.sort(key=lambda r: r[1])
    return rows


def short(name):
    n = name.replace("sgcn::(anonymous namespace)::", "")
    if n.startswith("void "):
        n = n[5:]
    i = n.find("(")
    return n[:i] if i > 0 else n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--csv", default=None)
    ap.add_argument("--timeline", action="store_true")
    ap.add_argument("--marker", default="multi_tensor_apply",
                    help="substring of the first kernel of each optimizer step")
    a = ap.parse_args()
    rows = load(a.path)
    tot = OrderedDict()
    for name, s, e, _ in rows:
        d = tot.setdefault(name, [0, 0])
        d[0] += 1
        d[1] += e - s
    alltime = sum(v[1] for v in tot.values())
    items = sorted(tot.items(), key=lambda kv: -kv[1][1])
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
            for n, (cnt, t) in items:
                w.writerow([n, cnt, t, f"{t / cnt:.1f}", f"{100.0 * t / alltime:.2f}"])
    for n, (cnt, t) in items[:40]:
        print(f"{100.0 * t / alltime:6.2f}% {cnt:5d} {t / cnt / 1e3:9.1f}us  {short(n)[:110]}")
    if a.timeline:
        idx = [i for i, r in enumerate(rows) if a.marker in r[0]]
        # the optimizer may launch several kernels: keep the first of each run
        starts = [i for k, i in enumerate(idx) if k == 0 or idx[k - 1] != i - 1]
        if len(starts) < 2:
            print("no step marker found", file=sys.stderr)
            return
        lo, hi = starts[-2], starts[-1]
        # step = dispatches after the previous optimizer run through this one
        while lo < hi and a.marker in rows[lo][0]:
            lo += 1
        while hi < len(rows) and a.marker in rows[hi][0]:
            hi += 1
        step = rows[lo:hi]
        busy = sum(e - s for _, s, e, _ in step)
        wall = step[-1][2] - step[0][1]
        print(f"\nlast step: {len(step)} dispatches, busy {busy / 1e6:.3f} ms, "
              f"wall {wall / 1e6:.3f} ms")
        for name, s, e, g in step:
            print(f"{(e - s) / 1e3:9.1f}us  {short(name)[:100]}  {g}")


if __name__ == "__main__":
    main()
