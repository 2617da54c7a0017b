"""Summarise SQ counter passes (tools/bench/pmc_pw.sh) per kernel+grid."""
import collections
import csv
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_pw"
rows = collections.OrderedDict()
for p in ("p1", "p2", "p3"):
    with open(f"{d}/{p}/run_counter_collection.csv") as f:
        for r in csv.DictReader(f):
            k = (p, r["Dispatch_Id"])
            e = rows.setdefault(k, {"name": r["Kernel_Name"], "grid": r["Grid_Size"],
                                    "dur": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
            e[r["Counter_Name"]] = float(r["Counter_Value"])
agg = collections.OrderedDict()
for (p, _), v in rows.items():
    n = v["name"].replace("sgcn::(anonymous namespace)::", "").replace("void ", "")
    n = n[:n.find("(")] if "(" in n else n
    a = agg.setdefault((n, v["grid"]), collections.defaultdict(list))
    for c, x in v.items():
        if c not in ("name", "grid"):
            a[c].append(x)
for (n, g), a in agg.items():
    m = {c: sum(x) / len(x) for c, x in a.items()}
    gui = m.get("GRBM_GUI_ACTIVE", 0)
    simd_cyc = gui * 256 * 4
    wc = m.get("SQ_WAVE_CYCLES", 1)
    print(f"{n[:70]} grid={g} dur={m['dur']/1e3:.1f}us")
    print("   mfma_busy/(gui*1024)=%.2f  waves: wait_any %.2f wait_inst %.2f active %.2f (valu %.2f lds %.2f vmem %.2f)" % (
        m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(1, simd_cyc), m.get("SQ_WAIT_ANY", 0) / wc,
        m.get("SQ_WAIT_INST_ANY", 0) / wc, m.get("SQ_ACTIVE_INST_ANY", 0) / wc,
        m.get("SQ_ACTIVE_INST_VALU", 0) / wc, m.get("SQ_ACTIVE_INST_LDS", 0) / wc,
        m.get("SQ_ACTIVE_INST_VMEM", 0) / wc))
    print("   per-mfma: valu %.2f lds %.2f vmem_rd %.2f vmem_wr %.2f salu %.2f | bankconf/lds %.2f  avg waves/CU %.1f  TA fifo full %.0f" % (
        *(m.get(c, 0) / max(1, m.get("SQ_INSTS_MFMA", 1)) for c in
          ["SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SALU"]),
        m.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, m.get("SQ_INSTS_LDS", 1)),
        m.get("SQ_LEVEL_WAVES", 0) / max(1, m.get("SQ_CYCLES", 1)) / 256 * 4,
        m.get("SQ_VMEM_TA_ADDR_FIFO_FULL", 0)))
    print("   raw: mfma_busy %.3g gui %.3g insts_mfma %.3g wave_cycles %.3g busy_cycles %.3g" % (
        m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0), gui, m.get("SQ_INSTS_MFMA", 0), wc, m.get("SQ_BUSY_CYCLES", 0)))
