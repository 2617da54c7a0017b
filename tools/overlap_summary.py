"""Per-step view of a rocprofv3 kernel trace (kernel_trace.csv) of bench.py: for every
training step (delimited by the optimizer's launch) the wall time, the
busy time (union of kernel intervals), the summed kernel time per hardware queue (the
side-stream weight gradients run on their own queue), and, for the last step that used
more than one queue, the per-kernel-class sums.

    python tools/overlap_summary.py <kernel_trace.csv> [...]
"""
import collections
import csv
import sys


def short(n):
    n = n.replace("sgcn::(anonymous namespace)::", "")
    if n.startswith("void "):
        n = n[5:]
    i = n.find("(")
    n = n[:i] if i > 0 else n
    i = n.find("<")
    return n[:i] if i > 0 else n


def union(iv):
    iv = sorted(iv)
    busy, (cs, ce) = 0, iv[0]
    for s, e in iv[1:]:
        if s > ce:
            busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return busy + ce - cs


def main():
    for p in sys.argv[1:]:
        rows = sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                        r["Queue_Id"]) for r in csv.DictReader(open(p))), key=lambda r: r[1])
        # the optimizer's launch ends a step (FusedSGD: sgd_step_kernel; torch's SGD: its
        # first multi-tensor kernel)
        marks = [i for i, r in enumerate(rows) if "sgd_step_kernel" in r[0]]
        if not marks:
            marks = [i for i, r in enumerate(rows) if "multi_tensor_apply" in r[0]]
        starts = [marks[0]] + [m for a, m in zip(marks, marks[1:]) if m - a > 5]
        print(p)
        last_multi = None
        for a, b in zip(starts, starts[1:]):
            seg = rows[a + 1:b + 1]
            q = collections.defaultdict(float)
            for r in seg:
                q[r[3]] += (r[2] - r[1]) / 1e6
            wall = (max(r[2] for r in seg) - min(r[1] for r in seg)) / 1e6
            busy = union([(r[1], r[2]) for r in seg]) / 1e6
            print(f"  step: {len(seg)} dispatches  wall {wall:.3f} ms  busy {busy:.3f} ms  "
                  f"per-queue kernel ms {{{', '.join(f'{k}: {v:.3f}' for k, v in sorted(q.items()))}}}")
            if len(q) > 1:
                last_multi = seg
        if last_multi:
            cls = collections.defaultdict(float)
            for r in last_multi:
                cls[short(r[0])] += (r[2] - r[1]) / 1e6
            print("  last multi-queue step, kernel ms by class:")
            for k, v in sorted(cls.items(), key=lambda kv: -kv[1])[:16]:
                print(f"    {k:30s} {v:.3f}")


if __name__ == "__main__":
    main()
