"""Per-kernel HBM traffic from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

    python tools/pmc_summary.py <pmc_dir> [--match SUBSTR] [--json OUT --tag NAME]

--json writes the HBM bytes per C-ABI call of each launch-timer op class (bench.py's
roofline classes; an op's helper kernels, e.g. pw_dw's slab reduce, count with it),
which bench.py reports as roofline.traffic for the dominant class.

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


# op class (ops.LaunchTimer name) -> (primary kernel prefixes, helper kernel prefixes). The
# primary kernels count the C-ABI calls; every kernel of the class adds to its bytes.
OP_CLASSES = {
    "pw_fwd": (("pwg_fwd_kernel", "pw_fwd_smallm_kernel"), ("tshift_params_kernel",)),
    "pw_dw": (("pw_dw_kernel", "pw_dw3_kernel", "pw_dw_smallc_kernel"), ("slab_reduce_kernel",)),
    "tshift_fwd": (("tshift_fwd_kernel", "tshift_fwd_lds_kernel", "tshift_fwd_pad_kernel",
                    "tshift_fwd_pre_kernel", "tshift_fwd_tail_kernel"), ()),
    "tshift_bwd": (("tshift_bwd_kernel", "tshift_bwd_ra_kernel", "tshift_bwd_s2_kernel"), ()),
    "bn_stats": (("moments_kernel", "moments_ja_kernel"), ()),
    "bn_apply": (("bn_apply_kernel", "bn_apply_ja_kernel"), ()),
    "bn_bwd_reduce": (("bn_bwd_reduce_kernel", "bn_bwd_reduce_ja_kernel"), ()),
    "bn_bwd_apply": (("bn_bwd_apply_kernel", "bn_bwd_apply_ja_kernel"), ()),
    "gcn_dx_finish": (("gcn_dx_finish_kernel", "gcn_dx_finish_ja_kernel"), ()),
    "gcn_gather": (("gcn_gather_kernel",), ()),
    "finalize": (("bn_finalize_kernel", "bn_eval_coef_kernel", "bn_bwd_finalize_kernel",
                  "bn_bwd_finalize_gbn_kernel", "mask_prep_kernel", "mask_grad_finalize_kernel",
                  "tshift_pos_finalize_kernel"), ()),
    "head": (("head_moments_kernel", "head_apply_kernel", "head_bwd_reduce_kernel",
              "head_bwd_apply_kernel", "modalities_kernel"), ()),
    "pool": (("pool_kernel", "pool_bwd_kernel"), ()),
}
# FETCH_SIZE correction per kernel: x2 for reads whose wave instructions cover whole 128-B
# lines (calibrated with known-byte kernels: profiles/r02_calib, profiles/r03_fetchcal); the
# split-K pw_dw3 weight-gradient kernels stage 16 positions per operand row per wave
# instruction (64-B row segments), for which the counter is NOT calibrated
# (tools/bench/fetchcal: 0.52x-1.09x of the true bytes raw): reported raw, i.e. a lower
# bound, with the x2 figure as the upper bound (fetch_bytes_x2_upper).
UNCALIBRATED = ("pw_dw3_kernel",)


def op_traffic(f, w, iters=0):
    """{op: {calls, fetch_bytes, write_bytes, bytes_per_call[, bytes_per_step]}}."""
    out = {}
    for op, (prim, helpers) in OP_CLASSES.items():
        calls, fb, fbu, wb = 0, 0.0, 0.0, 0.0
        for (n, _, fv, _), (_, _, wv, _) in zip(f, w):
            k = short(n)
            if k.startswith(prim):
                calls += 1
            elif not (helpers and k.startswith(helpers)):
                continue
            fb += fv if k.startswith(UNCALIBRATED) else 2 * fv
            fbu += 2 * fv
            wb += wv
        if calls:
            d = {"calls": calls, "fetch_bytes": fb / calls, "write_bytes": wb / calls,
                 "bytes_per_call": (fb + wb) / calls}
            if fbu != fb:
                d["fetch_bytes_x2_upper"] = fbu / calls
                d["bytes_per_call_upper"] = (fbu + wb) / calls
            if iters:
                d["calls_per_step"] = calls / iters
                d["bytes_per_step"] = (fb + wb) / iters
            out[op] = d
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--match", default="")
    ap.add_argument("--json", default="")
    ap.add_argument("--tag", default="")
    ap.add_argument("--iters", type=int, default=0,
                    help="steps (or ensemble iterations) the traced run executed: per-step bytes")
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
    if a.json:
        import json
        ops = op_traffic(f, w, a.iters)
        with open(a.json, "w") as fh:
            json.dump({"source": a.tag or a.dir,
                       "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate "
                                 "kernel-trace passes over bench.py --steps 2 --warmup 1 "
                                 "(serialized schedule); FETCH_SIZE doubled (gfx950 wide-read "
                                 "correction) except for the uncalibrated 64-/128-B row-segment "
                                 "reads of the weight-gradient kernels (raw; x2 as "
                                 "fetch_bytes_x2_upper), WRITE_SIZE as is (MI355X_MICROARCH.md "
                                 "HBM section); per C-ABI call and per step",
                       "iters": a.iters, "ops": ops}, fh, indent=1)
        for k, v in ops.items():
            print(f"{k:14s} calls={v['calls']:4d} bytes/call={v['bytes_per_call'] / 1e6:9.1f} MB")


if __name__ == "__main__":
    main()
