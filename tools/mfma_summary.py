"""MFMA utilisation per contraction instantiation from a rocprofv3 SQ counter pass over
the training step (tools/gpu_pmc_round.sh):

    python tools/mfma_summary.py <dir-with-run_counter_collection.csv>

util = SQ_VALU_MFMA_BUSY_CYCLES / (SIMD-cycles of the dispatch): MFMA_BUSY counts 64
cycles per v_mfma_f32_32x32x2_f32 summed over all SIMDs (checked: busy / insts = 64), and
GRBM_GUI_ACTIVE sums the active GPU clocks of the 8 XCDs, so the dispatch offers
GUI/8 x 1024 SIMD-cycles (256 CUs x 4 SIMDs). VALU per MFMA shows the issue-slot
competition (on gfx950 the fp32 MFMA and the VALU share the issue: DESIGN.md).
"""
import collections
import csv
import os
import sys

d = sys.argv[1]
path = os.path.join(d, "run_counter_collection.csv")
rows = collections.OrderedDict()
with open(path) as f:
    for r in csv.DictReader(f):
        e = rows.setdefault(r["Dispatch_Id"], {"name": r["Kernel_Name"], "grid": r["Grid_Size"],
                                              "dur": int(r["End_Timestamp"]) -
                                              int(r["Start_Timestamp"])})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
agg = collections.OrderedDict()
for v in rows.values():
    n = v["name"].replace("sgcn::(anonymous namespace)::", "").replace("void ", "")
    n = n[:n.find("(")] if "(" in n else n
    if not n.startswith(("pwg_fwd_kernel", "pw_dw3_kernel", "pw_dw_kernel")):
        continue
    a = agg.setdefault((n, v["grid"]), collections.defaultdict(list))
    for c, x in v.items():
        if c not in ("name", "grid"):
            a[c].append(x)
print(f"{'kernel':72s} {'grid':>9s} {'n':>3s} {'us':>7s} {'util':>5s} {'valu/mfma':>9s} "
      f"{'busy/64':>8s}")
tot_busy = tot_avail = 0.0
for (n, g), a in sorted(agg.items(), key=lambda kv: -sum(kv[1]["dur"])):
    m = {c: sum(x) / len(x) for c, x in a.items()}
    avail = m.get("GRBM_GUI_ACTIVE", 0) / 8 * 1024
    busy = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)
    insts = max(1.0, m.get("SQ_INSTS_MFMA", 1))
    tot_busy += busy * len(a["dur"])
    tot_avail += avail * len(a["dur"])
    print(f"{n[:72]:72s} {g:>9s} {len(a['dur']):3d} {m['dur'] / 1e3:7.1f} "
          f"{busy / max(1.0, avail):5.2f} {m.get('SQ_INSTS_VALU', 0) / insts:9.2f} "
          f"{busy / insts / 64:8.2f}")
print(f"all contraction dispatches: MFMA busy {tot_busy / max(1.0, tot_avail):.3f} of their "
      "SIMD-cycles")
