"""Compare two rocprofv3 kernel_stats.csv files by kernel class (ms per step)."""
import collections
import csv
import re
import sys


def load(f, steps):
    d = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        m = re.search(r'(\w+_kernel)', r['Name'])
        k = m.group(1) if m else r['Name'][:40]
        d[k] += float(r['TotalDurationNs']) / steps / 1e6
    return d


if __name__ == "__main__":
    steps = float(sys.argv[3]) if len(sys.argv) > 3 else 7
    A, B = load(sys.argv[1], steps), load(sys.argv[2], steps)
    for k in sorted(set(A) | set(B), key=lambda k: -max(A.get(k, 0), B.get(k, 0)))[:18]:
        print(f"{k:35s} {A.get(k, 0):7.2f} {B.get(k, 0):7.2f} {B.get(k, 0) - A.get(k, 0):+7.2f}")
    print(f"{'total':35s} {sum(A.values()):7.2f} {sum(B.values()):7.2f}")
