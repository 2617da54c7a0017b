"""Shift-GCN training throughput on MI355X: skeleton clips/s, fwd+bwd (+SGD step).

BASELINE.json metric: "skeleton clips/sec fwd+bwd, NTU (3,300,25,2) bs=64; 1/2/4/8 MI355X".
One step = one reference training iteration (main.py:397-416) on one synthetic NTU batch
per GPU: Model forward (10 fused TCN_GCN_units on the HIP path), CrossEntropy, backward,
[RCCL gradient all-reduce for N>1], SGD(momentum 0.9, nesterov, per-param weight decay).
Inputs are resident in HBM before the timed region. Weak scaling: 64 clips per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config ntu|mp|ens] [--graph 0|1]
--config ens: BASELINE config 4 instead (4-stream MediaPipe ensemble inference, bs=256,
eval mode, one hipGraph per batch): windows/s, its own JSON line.
N>1: `python bench.py --gpus N` starts N ranks itself (one process per GPU, through
torch.distributed.run as a child process, before anything touches a GPU), or run it under
an explicit launcher: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N;
a launcher's WORLD_SIZE that differs from --gpus is an error (exit 2).

Prints ONE JSON line on rank 0 (value = whole-job clips/s), with:
  roofline     — dominant kernel class of the timed region, achieved algorithmic
                 FLOP/s (or bytes/s) from HIP events around every launch of it;
  cpu_baseline — the PyTorch-eager CPU restatement (oracle/, "port") on the host cores,
                 on a bounded sample (2 clips, fwd+bwd+SGD), rank 0 / N=1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(REPO, "shift-gcn_amd"), REPO):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

CONFIGS = {
    # name: (num_class, V, M, T, graph)
    "ntu": (60, 25, 2, 300, "graph.ntu_rgb_d.Graph"),
    "mp": (2, 33, 1, 300, "graph.mediapipe_pose.Graph"),
}
# algorithmic fwd+bwd GFLOP per clip (torch FlopCounter on the reference model)
GFLOP_PER_CLIP = {"ntu": 21.416, "mp": 14.134}
GFLOP_PER_WINDOW_ENS = 18.85   # 4 MediaPipe forwards per window
PEAK_FP32_TFLOPS = 157.3   # MI355X FP32 matrix (= vector) dense peak, MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0      # HBM3E spec
# HBM bytes per C-ABI call of each op class from the committed rocprofv3 PMC passes
# (tools/pmc_traffic.sh + tools/pmc_summary.py --json) of this code version
PMC_TRAFFIC = os.path.join(REPO, "profiles", "pmc_traffic.json")
# per-config PMC files (the NTU figures must never be quoted on another workload)
PMC_TRAFFIC_BY_CONFIG = {"ntu": PMC_TRAFFIC,
                         "mp": os.path.join(REPO, "profiles", "pmc_traffic_mp.json")}
PMC_TRAFFIC_ENS = os.path.join(REPO, "profiles", "pmc_traffic_ens.json")


def pmc_traffic(op, path=None):
    try:
        with open(path or PMC_TRAFFIC) as f:
            d = json.load(f)
        return d["ops"][op]["bytes_per_call"], d.get("source", "")
    except (OSError, KeyError, ValueError):
        return None, ""


def pmc_ops(path):
    try:
        with open(path) as f:
            return json.load(f).get("ops", {})
    except (OSError, ValueError):
        return {}


def class_rates(summ, n_iters, pmc=None):
    """Per op class: ms per step and the achieved rate against its own bound — TF/s of
    algorithmic FLOP vs the FP32 MFMA peak for the contractions, GB/s of algorithmic bytes
    vs the HBM peak for the streaming passes (SURVEY §8d per-kernel definitions) — plus the
    HBM bytes per step the committed PMC passes measured for the class, when present."""
    out = {}
    for k, v in sorted(summ.items()):
        sec = v["ms_total"] / 1e3
        e = {"ms": round(v["ms_total"] / n_iters, 3), "launches": v["launches"] // n_iters}
        gbs = v["bytes"] / sec / 1e9 if sec > 0 else 0.0
        if v["flops"] > 0:
            tf = v["flops"] / sec / 1e12 if sec > 0 else 0.0
            e.update(bound="mfma", tflops=round(tf, 2), frac=round(tf / PEAK_FP32_TFLOPS, 4),
                     gbs_algorithmic=round(gbs, 1))
        else:
            e.update(bound="hbm", gbs=round(gbs, 1), frac=round(gbs / PEAK_HBM_GBS, 4))
        e["algorithmic_mb_per_step"] = round(v["bytes"] / n_iters / 1e6, 1)
        t = (pmc or {}).get(k, {})
        if "bytes_per_step" in t:
            e["pmc_mb_per_step"] = round(t["bytes_per_step"] / 1e6, 1)
            if v["bytes"] > 0:
                e["pmc_over_algorithmic"] = round(t["bytes_per_step"] / (v["bytes"] / n_iters), 3)
        out[k] = e
    return out


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=None,
                    help="clips (windows for --config ens) per GPU; default 64 (ens: 256)")
    ap.add_argument("--config", default="ntu", choices=sorted(CONFIGS) + ["ens"])
    ap.add_argument("--graph", type=int, default=0, help="capture the step in a hipGraph")
    ap.add_argument("--graph-ens", type=int, default=1,
                    help="--config ens: replay the ensemble forward as one hipGraph")
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--roofline", type=int, default=1)
    ap.add_argument("--data", default=None,
                    help="on-disk (N,3,T,V,M) float32 .npy clips (feeders/feeder.py format), "
                         "memory-mapped and streamed to the GPU by shiftgcn.feeder; default: "
                         "one synthetic batch resident in HBM")
    ap.add_argument("--labels", default=None, help="(sample_name, label) pickle for --data")
    return ap.parse_args()


def host_threads():
    """(threads used, affinity cores): every core of this process's CPU share. The GPU box
    grants each GPU a share of the host (OMP_NUM_THREADS, 16 per GPU there) while
    sched_getaffinity shows the whole machine, so the share caps the affinity set."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    share = os.environ.get("OMP_NUM_THREADS")
    n = aff if not share or not share.isdigit() else max(1, min(aff, int(share)))
    return n, aff


def cpu_baseline(cfg, seconds_budget=30.0):
    """The oracle (PyTorch-eager CPU restatement of the reference model with the naive
    torch-gather temporal shift, oracle/torch_shift.py) on the host cores, bounded samples
    of the same workload:
      * the metric's unit: 2 clips fwd+bwd+SGD (median of 3 after 1 warm-up);
      * BASELINE config 1: NTU bs=2 forward only (median of >= 5 after 1 warm-up)."""
    from oracle import model_oracle as mo
    from oracle import torch_shift as ts
    num_class, V, M, T, _ = CONFIGS[cfg]
    threads, ncpu = host_threads()
    prev = torch.get_num_threads()
    prev_fn = mo.Shift.function
    torch.set_num_threads(threads)
    mo.Shift.function = ts.TorchShiftFunction    # torch.gather shift (config 1's fallback)
    try:
        torch.manual_seed(1)
        model = mo.Model(num_class=num_class, num_point=V, num_person=M, graph="unused").train()
        opt = torch.optim.SGD(mo.sgd_param_groups(model, 0.1), lr=0.1, momentum=0.9,
                              nesterov=True)
        g = torch.Generator().manual_seed(0)
        n = 2
        x = torch.randn(n, 3, T, V, M, generator=g)
        y = torch.randint(0, num_class, (n,), generator=g)

        def it():
            loss = torch.nn.functional.cross_entropy(model(x), y)
            opt.zero_grad()
            loss.backward()
            opt.step()

        it()  # warm-up
        times = []
        t_all = time.perf_counter()
        while len(times) < 3 and time.perf_counter() - t_all < seconds_budget:
            t0 = time.perf_counter()
            it()
            times.append(time.perf_counter() - t0)
        times.sort()
        med = times[len(times) // 2]
        # BASELINE config 1: NTU x-sub joint, bs=2, Model forward on CPU PyTorch eager
        fwd = None
        if cfg == "ntu":
            model.eval()
            with torch.no_grad():
                model(x)
                ft = []
                t_all = time.perf_counter()
                while len(ft) < 5 or (len(ft) < 7 and time.perf_counter() - t_all < 10):
                    t0 = time.perf_counter()
                    model(x)
                    ft.append(time.perf_counter() - t0)
            model.train()
            ft.sort()
            fmed = ft[len(ft) // 2]
            fwd = {"value": round(n / fmed, 4), "unit": "clips/s", "s_per_iter": round(fmed, 4),
                   "runs": len(ft), "cores": threads,
                   "sample": "BASELINE config 1: NTU bs=2 (2,3,300,25,2) Model forward "
                             "(eval, no_grad), median of runs after 1 warm-up"}
        model_name = ""
        try:
            with open("/proc/cpuinfo") as f:
                for line in f:
                    if line.startswith("model name"):
                        model_name = line.split(":", 1)[1].strip()
                        break
        except OSError:
            pass
        return {"value": round(n / med, 4), "unit": "clips/s", "cores": threads,
                "kind": "port",
                "sample": f"{cfg.upper()} bs={n} (2 clips of the bs=64 workload), fwd+bwd+SGD, "
                          f"median of {len(times)} after 1 warm-up, {med:.2f} s/iter; "
                          f"{threads} threads = this process's CPU share ({ncpu} cores in "
                          f"its affinity set); {model_name}",
                "config1_forward": fwd}
    finally:
        torch.set_num_threads(prev)
        mo.Shift.function = prev_fn


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_command(argv, n, port):
    """The child command that runs this benchmark on ``n`` ranks of this node (one process
    per GPU, rendezvous on 127.0.0.1): the same arguments, under torch.distributed.run."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={n}", "--master-addr=127.0.0.1", f"--master-port={port}",
            os.path.abspath(__file__)] + list(argv)


def check_world(gpus, env):
    """World size this process must run at: ``--gpus`` when no launcher set WORLD_SIZE
    (None = start the ranks first), else the launcher's, which must equal ``--gpus``."""
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return None if gpus > 1 else 1
    if int(ws) != gpus:
        raise SystemExit(2)
    return int(ws)


def main():
    args = parse()
    if args.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr)
        raise SystemExit(2)
    try:
        world = check_world(args.gpus, os.environ)
    except SystemExit:
        print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE="
              f"{os.environ.get('WORLD_SIZE')} ranks", file=sys.stderr)
        raise
    if world is None:
        # --gpus N without a launcher: start the N ranks as a child process (nothing in this
        # process has touched a GPU), relay their output, exit with their status
        import subprocess
        have = torch.cuda.device_count()   # (does not initialise a device on this image)
        if have < args.gpus and os.environ.get("SGCN_BENCH_SAME_DEVICE") != "1":
            print(f"bench.py: --gpus {args.gpus} but {have} GPUs are visible", file=sys.stderr)
            raise SystemExit(2)
        cmd = launch_command(sys.argv[1:], args.gpus, _free_port())
        raise SystemExit(subprocess.call(cmd))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1
    # Rehearsal knobs (never set by the driver): SGCN_BENCH_BACKEND=gloo and
    # SGCN_BENCH_SAME_DEVICE=1 run N ranks on one GPU to exercise the N>1 code path.
    backend = os.environ.get("SGCN_BENCH_BACKEND", "nccl")
    if os.environ.get("SGCN_BENCH_SAME_DEVICE") == "1":
        local = 0
    if distributed:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    if args.config == "ens":
        return bench_ensemble(args, dev, rank, world, distributed)
    if args.batch is None:
        args.batch = 64

    import shiftgcn
    from shiftgcn import ops, train
    from shiftgcn.dist import GradAllReduce, broadcast_parameters

    num_class, V, M, T, graph = CONFIGS[args.config]
    torch.manual_seed(1)                                # main.py:24-27 init seed
    model = shiftgcn.Model(num_class=num_class, num_point=V, num_person=M, graph=graph)
    model = model.to(dev).train()
    if distributed:
        broadcast_parameters(model)
    opt = train.build_optimizer(model, base_lr=0.1)
    # N>1: the gradients are written into the all-reduce bucket by the backward and the
    # 1/world is applied inside the one-launch optimizer update: one all-reduce + one update
    # launch between backward() and the next step (shiftgcn.dist.GradAllReduce)
    sync = None
    if distributed:
        sync = GradAllReduce(model, defer_scale_to=opt if isinstance(opt, train.FusedSGD)
                             else None)
    gen = torch.Generator().manual_seed(1000 + rank)
    x = torch.randn(args.batch, 3, T, V, M, generator=gen).to(dev)
    label = torch.randint(0, num_class, (args.batch,), generator=gen).to(dev)
    batches = None
    if args.data:
        # real clips: mmap -> pinned staging -> H2D on a copy stream, one batch ahead of
        # the step (shiftgcn.feeder.DeviceBatchLoader); epochs repeat as needed
        from shiftgcn.feeder import DeviceBatchLoader, Feeder
        if not args.labels:
            raise SystemExit("--data needs --labels")
        if args.graph:
            raise SystemExit("--data feeds a new batch every step: run it without --graph")
        feeder = Feeder(args.data, args.labels)
        if tuple(feeder.data.shape[1:]) != (3, T, V, M):
            raise SystemExit(f"--data clips are {feeder.data.shape[1:]}, config "
                             f"{args.config} needs (3, {T}, {V}, {M})")
        loader = DeviceBatchLoader(feeder, args.batch, shuffle=True, drop_last=True,
                                   device=dev, rank=rank, world_size=world)
        if len(loader) == 0:
            raise SystemExit("--data holds fewer clips than one global batch")

        def _stream():
            while True:
                yield from loader
        batches = _stream()

    def step():
        if batches is not None:
            xb, yb, _ = next(batches)
            return train.train_step(model, opt, xb, yb, grad_sync=sync)
        return train.train_step(model, opt, x, label, grad_sync=sync)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    runner = step
    if args.graph:
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            step()
        torch.cuda.current_stream().wait_stream(s)
        with torch.cuda.graph(g):
            step()
        runner = g.replay

    if sync is not None and not args.graph:
        sync.timing(True)   # HIP events around each timed step's all_reduce
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        runner()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    rank_ms = [round(1000.0 * elapsed / args.steps, 3)]
    if distributed:
        elapsed, rank_ms = _max_over_ranks(elapsed, dev, world, args.steps)
    comm = None
    if sync is not None:
        comm = sync.timing_summary()
        sync.timing(False)
        comm["allreduce_ms_per_step_max_over_ranks"] = (
            None if comm["allreduce_ms_per_step"] is None else
            _max_over_ranks(comm["allreduce_ms_per_step"], dev, world, 1)[0])

    clips = args.batch * world * args.steps
    value = clips / elapsed
    ms = 1000.0 * elapsed / args.steps

    roof = None
    if args.roofline:
        # HIP events around every launch of each kernel class, over K eager steps. Every
        # rank runs these steps (they contain the gradient all-reduce, so a rank-0-only
        # loop would wait forever for the others); rank 0 reports.
        # The timed steps run the weight-gradient contractions on a side stream, overlapped
        # with the input-gradient chain (shiftgcn.fused._OffPath); concurrent kernels share
        # the CUs, so a per-launch duration there is not the kernel's own rate. These steps
        # run serialized (side stream off) so every class is timed alone.
        from shiftgcn import fused
        async_dw = fused.ASYNC_DW
        fused.ASYNC_DW = 0
        timer = ops.LaunchTimer()
        ops.set_launch_timer(timer)
        torch.cuda.synchronize()
        n_meas = max(1, min(args.steps, 5))
        s0 = torch.cuda.Event(enable_timing=True)
        s1 = torch.cuda.Event(enable_timing=True)
        s0.record()
        for _ in range(n_meas):
            step()
        s1.record()
        torch.cuda.synchronize()
        ops.set_launch_timer(None)
        fused.ASYNC_DW = async_dw
        step_ms_meas = s0.elapsed_time(s1) / n_meas
        summ = timer.summary()
        dom = max(summ, key=lambda k: summ[k]["ms_total"])
        d = summ[dom]
        mfma = d["flops"] > 0
        per_launch_s = d["ms_total"] / d["launches"] / 1e3
        if mfma:
            achieved = d["flops"] / d["launches"] / per_launch_s / 1e12
            peak, unit = PEAK_FP32_TFLOPS, "TFLOP/s"
        else:
            achieved = d["bytes"] / d["launches"] / per_launch_s / 1e9
            peak, unit = PEAK_HBM_GBS, "GB/s"
        traffic, tsrc = pmc_traffic(dom, PMC_TRAFFIC_BY_CONFIG.get(args.config))
        roof = {"bound": "mfma" if mfma else "hbm", "kernel": dom,
                "achieved": round(achieved, 3), "peak": peak, "unit": unit,
                "frac": round(achieved / peak, 4),
                # per launch max(FLOP/157.3T, bytes/8T) summed, over the measured time: the
                # fraction of its own roofline (MFMA- or HBM-bound per launch) the class runs at
                "roofline_time_frac": round(d["roof_ms"] / d["ms_total"], 4),
                "timed_classes_roofline_time_frac": round(
                    sum(v["roof_ms"] for v in summ.values()) /
                    sum(v["ms_total"] for v in summ.values()), 4),
                "traffic": None if traffic is None else round(traffic),
                "traffic_unit": "HBM bytes per launch (PMC FETCH_SIZE x2 + WRITE_SIZE)",
                "traffic_source": tsrc or None,
                "algorithmic_bytes_per_launch": round(d["bytes"] / d["launches"]),
                "launches_per_step": d["launches"] // n_meas,
                "avg_launch_us": round(per_launch_s * 1e6, 2),
                "step_breakdown_ms": {k: round(v["ms_total"] / n_meas, 3)
                                      for k, v in sorted(summ.items())},
                "class_rates": class_rates(
                    summ, n_meas, pmc_ops(PMC_TRAFFIC_BY_CONFIG.get(args.config, ""))),
                # HIP events around every C-ABI launch vs events around the whole step (same
                # steps): the rest is torch's head/loss/optimizer kernels and launch gaps
                "step_ms_event_timed": round(step_ms_meas, 3),
                "step_other_ms": round(step_ms_meas - sum(v["ms_total"] for v in summ.values())
                                       / n_meas, 3),
                "breakdown_coverage": round(sum(v["ms_total"] for v in summ.values())
                                            / n_meas / step_ms_meas, 4),
                "whole_step_frac_of_fp32_peak": round(
                    value / world * GFLOP_PER_CLIP[args.config] / 1e3 / PEAK_FP32_TFLOPS, 4),
                # context for the HBM-bound classes: what a plain copy of one activation
                # (read + write, plain stores) reaches on this box in this run
                "hbm_copy_gbs_measured": _copy_rate_gbs(dev, 4 * args.batch * M * 64 * T * V),
                "schedule": ("timed steps: weight gradients on a side stream"
                             if async_dw else "timed steps: serialized") +
                            "; roofline/breakdown steps: serialized (each class timed alone)"}

    cpu = None
    if args.cpu_baseline and rank == 0:   # after the timed region (the other ranks wait)
        cpu = cpu_baseline(args.config)

    if rank == 0:
        line = {
            "metric": "skeleton clips/sec fwd+bwd, NTU (3,300,25,2) bs=64; 1/2/4/8 MI355X"
            if args.config == "ntu" else
            "skeleton clips/sec fwd+bwd, MediaPipe (3,300,33,1) bs=64",
            "value": round(value, 2),
            "unit": "clips/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": (f"on-disk clips {os.path.basename(args.data)} (mmap, streamed to HBM "
                     "inside the timed region), random-init weights (seeded)" if args.data else
                     "synthetic N(0,1) clips, random-init weights (seeded)"),
            "config": {"workload": f"{args.config.upper()} Shift-GCN training step "
                                   f"(fwd+CE+bwd+SGD), x=({args.batch},3,{T},{V},{M}) per GPU",
                       "global_batch": args.batch * world, "per_gpu_batch": args.batch,
                       "parallelism": f"dp{world}", "hipgraph": bool(args.graph),
                       **_ranks_info(distributed, world, rank_ms), **_comm_info(comm)},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


def _copy_rate_gbs(dev, nbytes, reps=10):
    """Algorithmic GB/s of torch's copy_ of an nbytes fp32 tensor (read + write), event-timed:
    the box's achievable rate for a one-read-one-write stream (tools/bench/streambench.hip
    measures the hand-written forms: 5.0-5.8 TB/s, profiles/r05_dma/)."""
    x = torch.ones(nbytes // 4, device=dev)
    y = torch.empty_like(x)
    y.copy_(x)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        y.copy_(x)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    del x, y
    return round(2 * nbytes / ms / 1e6, 1)


def _max_over_ranks(elapsed, dev, world, steps):
    """(max over ranks of the timed region, every rank's ms per step in rank order)."""
    t = torch.zeros(world, device=dev, dtype=torch.float64)
    t[dist.get_rank()] = elapsed
    dist.all_reduce(t, op=dist.ReduceOp.SUM)   # each rank fills its own slot
    per = t.cpu().tolist()
    return max(per), [round(1000.0 * e / steps, 3) for e in per]


def _ranks_info(distributed, world, rank_ms):
    """What ran: the process group's size and backend as torch.distributed reports them
    (1 / "none" without one) and each rank's timed ms per step."""
    if distributed:
        ws, be = dist.get_world_size(), str(dist.get_backend())
        if ws != world:
            raise RuntimeError(f"process group has {ws} ranks, WORLD_SIZE={world}")
    else:
        ws, be = 1, "none"
    return {"world_size": ws, "backend": be, "rank_ms_per_step": rank_ms}


def _comm_info(comm):
    """The gradient all-reduce of the timed steps (N > 1): HIP-event ms per step on this
    rank and the max over ranks, the bucket's bytes and the bus GB/s (ring convention);
    nulls at N = 1 (no collective) or under --graph (no events inside the capture)."""
    if comm is None:
        return {"allreduce_ms_per_step": None, "bucket_bytes": None,
                "allreduce_bus_gbs": None}
    return {k: comm[k] for k in ("allreduce_ms_per_step", "allreduce_ms_per_step_max_over_ranks",
                                 "bucket_bytes", "allreduce_bus_gbs")}


def _roofline(summ, n_iters, value_per_gpu, gflop_per_unit):
    dom = max(summ, key=lambda k: summ[k]["ms_total"])
    d = summ[dom]
    mfma = d["flops"] > 0
    per_launch_s = d["ms_total"] / d["launches"] / 1e3
    if mfma:
        achieved = d["flops"] / d["launches"] / per_launch_s / 1e12
        peak, unit = PEAK_FP32_TFLOPS, "TFLOP/s"
    else:
        achieved = d["bytes"] / d["launches"] / per_launch_s / 1e9
        peak, unit = PEAK_HBM_GBS, "GB/s"
    return {"bound": "mfma" if mfma else "hbm", "kernel": dom,
            "achieved": round(achieved, 3), "peak": peak, "unit": unit,
            "frac": round(achieved / peak, 4), "traffic": None,
            "roofline_time_frac": round(d["roof_ms"] / d["ms_total"], 4),
            "algorithmic_bytes_per_launch": round(d["bytes"] / d["launches"]),
            "launches_per_iter": d["launches"] // n_iters,
            "avg_launch_us": round(per_launch_s * 1e6, 2),
            "iter_breakdown_ms": {k: round(v["ms_total"] / n_iters, 3)
                                  for k, v in sorted(summ.items())},
            "class_rates": class_rates(summ, n_iters, pmc_ops(PMC_TRAFFIC_ENS)),
            "whole_iter_frac_of_fp32_peak": round(
                value_per_gpu * gflop_per_unit / 1e3 / PEAK_FP32_TFLOPS, 4)}


def cpu_baseline_ensemble(seconds_budget=30.0):
    """The oracle ensemble (reference semantics: batch-1 forwards per window and stream,
    PyTorch eager on the host cores) on a bounded sample of 2 windows."""
    from oracle import ensemble_oracle as eo
    from oracle import model_oracle as mo
    from oracle import torch_shift as ts
    from shiftgcn.ensemble import MEDIAPIPE_BONE_PAIRS
    threads, _ = host_threads()
    prev = torch.get_num_threads()
    prev_fn = mo.Shift.function
    torch.set_num_threads(threads)
    mo.Shift.function = ts.TorchShiftFunction
    try:
        torch.manual_seed(1)
        models = {s: mo.Model(num_class=2, num_point=33, num_person=1, graph="unused").eval()
                  for s in eo.MODALITIES}
        g = torch.Generator().manual_seed(0)
        wins = [torch.randn(3, 300, 33, 1, generator=g).numpy() for _ in range(2)]
        eo.run_ensemble_inference(wins[:1], models, (0.6, 0.6, 0.4, 0.4), MEDIAPIPE_BONE_PAIRS)
        t0 = time.perf_counter()
        eo.run_ensemble_inference(wins, models, (0.6, 0.6, 0.4, 0.4), MEDIAPIPE_BONE_PAIRS)
        dt = time.perf_counter() - t0
        return {"value": round(len(wins) / dt, 4), "unit": "windows/s", "cores": threads,
                "kind": "port",
                "sample": f"2 MediaPipe windows (3,300,33,1), 4 streams, batch-1 forwards "
                          f"as inference_pipeline.py:355-366, {dt:.2f} s"}
    finally:
        torch.set_num_threads(prev)
        mo.Shift.function = prev_fn


def bench_ensemble(args, dev, rank, world, distributed):
    """BASELINE config 4: 4-stream (joint/bone/joint-motion/bone-motion) MediaPipe
    ensemble inference at bs=256 windows per GPU, eval mode, one hipGraph replay per
    batch. Replicas only across GPUs (inference has no exchange step)."""
    import shiftgcn
    from shiftgcn import ops
    from shiftgcn.ensemble import Ensemble, EnsembleGraph
    batch = args.batch or 256
    torch.manual_seed(1)
    models = [shiftgcn.Model(num_class=2, num_point=33, num_person=1,
                             graph="graph.mediapipe_pose.Graph").to(dev).eval()
              for _ in range(4)]
    ens = Ensemble(models).to(dev)
    gen = torch.Generator().manual_seed(2000 + rank)
    x = torch.randn(batch, 3, 300, 33, 1, generator=gen).to(dev)
    runner = (lambda: ens(x)) if not args.graph_ens else EnsembleGraph(ens, x.shape, dev).run
    call = (lambda: runner()) if not args.graph_ens else (lambda: runner(x))
    for _ in range(args.warmup):
        call()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        call()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    rank_ms = [round(1000.0 * elapsed / args.steps, 3)]
    if distributed:
        elapsed, rank_ms = _max_over_ranks(elapsed, dev, world, args.steps)
    value = batch * world * args.steps / elapsed
    roof = None
    if args.roofline and rank == 0:
        # eager, and with the four members in order (the timed iterations run them on four
        # streams: concurrent kernels share the CUs), so every class is timed alone
        from shiftgcn import ensemble as ens_mod
        ens_streams = ens_mod.ENS_STREAMS
        ens_mod.ENS_STREAMS = 0
        timer = ops.LaunchTimer()
        ops.set_launch_timer(timer)
        n = 3
        for _ in range(n):
            ens(x)
        torch.cuda.synchronize()
        ops.set_launch_timer(None)
        ens_mod.ENS_STREAMS = ens_streams
        roof = _roofline(timer.summary(), n, value / world, GFLOP_PER_WINDOW_ENS)
        roof["schedule"] = (("timed iterations: the four members on four streams"
                             if ens_streams else "timed iterations: members in order") +
                            "; roofline iterations: eager, members in order")
        traffic, tsrc = pmc_traffic(roof["kernel"], PMC_TRAFFIC_ENS)
        roof["traffic"] = None if traffic is None else round(traffic)
        roof["traffic_unit"] = "HBM bytes per launch (PMC FETCH_SIZE x2 + WRITE_SIZE)"
        roof["traffic_source"] = tsrc or None
    cpu = cpu_baseline_ensemble() if (args.cpu_baseline and rank == 0) else None
    if rank == 0:
        print(json.dumps({
            "metric": "ensemble windows/sec, MediaPipe 4-stream (3,300,33,1) bs=256 inference",
            "value": round(value, 2), "unit": "windows/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "fp32", "data": "synthetic N(0,1) windows, random-init weights (seeded)",
            "config": {"workload": f"ENS 4-stream eval forward + score fusion, "
                                   f"x=({batch},3,300,33,1) per GPU",
                       "global_batch": batch * world, "per_gpu_batch": batch,
                       "parallelism": f"replicas{world}", "hipgraph": bool(args.graph_ens),
                       **_ranks_info(distributed, world, rank_ms)},
            "roofline": roof, "cpu_baseline": cpu}), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
