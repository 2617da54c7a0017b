"""Config 5 (data-parallel training) semantics on ONE GPU, without a process group.

Two half-batch HIP forward/backward passes (what two ranks compute), combined with the
exact reduction GradAllReduce applies (``shiftgcn.dist.combine_local``: SUM over ranks x
the same per-element scale vector), against the single-process nn.DataParallel
restatement of the reference (``oracle/dp_oracle.py``, main.py:294-299) run on the CPU
oracle model in fp32 and fp64.

Bar (model-level fp32 gradients through 10 BatchNorm units are ill-conditioned, see
test_gpu_blocks.test_model_matches_golden_fixture): the HIP path is at least as close to the
fp64 DataParallel result as the fp32 DataParallel reference is (2x margin), logits and
running statistics within 1e-4, and no more ypos sign flips (vs fp64) than 2x the fp32
reference's + 2.

The multi-process RCCL path itself is unmeasured on hardware here (the driver runs the
8-GPU node); ``test_bench_two_ranks_same_device`` runs bench.py's N=2 code path (gloo
all-reduce, both ranks on cuda:0) to the JSON line.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

import formula
from conftest import REPO

pytestmark = pytest.mark.gpu
DEV = "cuda"
CFG = dict(N=4, T=24, V=25, M=2, num_class=60, seed=123)


def _inputs():
    x = formula.tensor((CFG["N"], 3, CFG["T"], CFG["V"], CFG["M"]), 77, 1.0)
    labels = torch.arange(CFG["N"]) * 7 % CFG["num_class"]
    return x, labels


def _oracle(dtype):
    from oracle import model_oracle as mo
    m = mo.Model(num_class=CFG["num_class"], num_point=CFG["V"], num_person=CFG["M"])
    formula.fill_state(m, seed=CFG["seed"])
    return m.to(dtype).train()


def _ours():
    import shiftgcn
    m = shiftgcn.Model(num_class=CFG["num_class"], num_point=CFG["V"], num_person=CFG["M"],
                       graph="graph.ntu_rgb_d.Graph")
    formula.fill_state(m, seed=CFG["seed"])
    return m.to(DEV).train()


def test_two_shard_hip_passes_match_dataparallel_emulation():
    from oracle.dp_oracle import dataparallel_grads
    from shiftgcn.dist import combine_local, trainable_named
    x, labels = _inputs()
    n = CFG["N"] // 2
    per_rank, models = [], []
    for r in range(2):
        m = _ours()
        out = m(x[r * n:(r + 1) * n].to(DEV))
        loss = torch.nn.functional.cross_entropy(out, labels[r * n:(r + 1) * n].to(DEV))
        m.zero_grad(set_to_none=True)
        loss.backward()
        per_rank.append({k: p.grad.detach().cpu() for k, p in trainable_named(m)})
        models.append((m, out.detach().cpu()))
    torch.cuda.synchronize()
    ours = combine_local(per_rank, trainable_named(models[0][0]))

    ref32, ref64 = _oracle(torch.float32), _oracle(torch.float64)
    _, logits32, g32 = dataparallel_grads(ref32, x, labels, 2)
    _, logits64, g64 = dataparallel_grads(ref64, x.double(), labels, 2)

    logits_ours = torch.cat([o for _, o in models]).double()
    scale = float(logits64.abs().max())
    assert float((logits_ours - logits64).abs().max()) <= 1e-4 * scale
    # rank 0 keeps its BatchNorm running statistics (DataParallel: replica 0's)
    b64 = dict(ref64.named_buffers())
    for k, b in models[0][0].named_buffers():
        if b.dtype.is_floating_point:
            ref = b64[k].double()
            err = float((b.double().cpu() - ref).abs().max())
            assert err <= 1e-4 * float(ref.abs().max()) + 1e-6, (k, err)

    names = sorted(g64)
    zero = [k.endswith(("Linear_bias", "down.0.bias", "residual.conv.bias")) for k in names]
    err_ours, err_ref, flips_ours, flips_ref = [], [], 0, 0
    for k, z in zip(names, zero):
        if k.endswith("ypos"):
            s64 = np.sign(g64[k].numpy())
            flips_ours += int((np.sign(ours[k].numpy()) != s64).sum())
            flips_ref += int((np.sign(g32[k].numpy()) != s64).sum())
            vals = set(np.round(ours[k].numpy() / 0.01).astype(int).tolist())
            assert vals <= {-2, 0, 2}, (k, vals)        # SUM of two +-0.01 replicas
            continue
        n64 = float(g64[k].norm())
        if z:
            assert float(ours[k].abs().max()) < 1e-3, k
            continue
        if n64 == 0.0:      # xpos: exactly 0 (the x-shift carries no gradient)
            assert float(ours[k].abs().max()) == 0.0, k
            continue
        err_ours.append(float((ours[k].double() - g64[k]).norm()) / n64)
        err_ref.append(float((g32[k].double() - g64[k]).norm()) / n64)
    err_ours, err_ref = np.array(err_ours), np.array(err_ref)
    assert np.median(err_ours) <= 2 * np.median(err_ref) + 1e-5, (np.median(err_ours),
                                                                   np.median(err_ref))
    assert err_ours.max() <= 2 * err_ref.max() + 1e-5, (err_ours.max(), err_ref.max())
    assert flips_ours <= 2 * flips_ref + 2, (flips_ours, flips_ref)


def test_bench_two_ranks_same_device():
    """``bench.py --gpus 2`` with no launcher starts its two ranks itself (one process per
    rank, GradAllReduce after backward, max-over-ranks timing, rank 0 prints) — here both on
    cuda:0 with a gloo all-reduce. The line records the process group torch.distributed
    reports (world size, backend) and every rank's ms per step. Also guards the
    rank-0-only-loop deadlock found in round 1 (every rank must run the roofline steps)."""
    env = dict(os.environ, SGCN_BENCH_BACKEND="gloo", SGCN_BENCH_SAME_DEVICE="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--batch", "4", "--cpu-baseline", "0"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 8 and d["value"] > 0
    assert d["config"]["world_size"] == 2 and d["config"]["backend"] == "gloo"
    rm = d["config"]["rank_ms_per_step"]
    assert len(rm) == 2 and abs(max(rm) - d["ms_per_step"]) < 1e-2, (rm, d["ms_per_step"])
    # the line explains its collective (HIP events around each timed
    # step's all_reduce, the bucket's bytes, the ring bus rate)
    c = d["config"]
    assert c["bucket_bytes"] == 4 * 693_107
    assert 0 < c["allreduce_ms_per_step"] <= c["allreduce_ms_per_step_max_over_ranks"]
    assert c["allreduce_ms_per_step_max_over_ranks"] < d["ms_per_step"]
    want = 2 * 1 / 2 * c["bucket_bytes"] / (c["allreduce_ms_per_step"] * 1e-3) / 1e9
    assert abs(c["allreduce_bus_gbs"] - want) <= 0.01 * want + 0.01


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("backend", ["gloo", "nccl"])
def test_gradients_are_written_into_the_bucket(backend):
    """Config 5's N>1 step (verdict r03): the HIP backward writes every trainable gradient
    straight into GradAllReduce's flat bucket, so the call copies nothing (one all-reduce,
    then the deferred 1/world inside the one-launch optimizer update). A world-1 group on the
    GPU — gloo, and RCCL (torch's "nccl" backend: the collective bench.py uses at N > 1, here
    with its one rank): every scale is 1 and the step must be bit-identical to the same step
    with no process group (no bucket, no slots)."""
    import torch.distributed as dist
    import shiftgcn  # noqa: F401
    from shiftgcn import train
    from shiftgcn.dist import GradAllReduce
    x, labels = _inputs()
    x, labels = x.to(DEV), labels.to(DEV)
    # reference: no data parallelism
    m_ref = _ours()
    o_ref = train.build_optimizer(m_ref, base_lr=0.1)
    for _ in range(2):
        train.train_step(m_ref, o_ref, x, labels)
    kw = {"device_id": torch.device(DEV, 0)} if backend == "nccl" else {}
    dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                            world_size=1, **kw)
    try:
        assert dist.get_backend() == backend
        m = _ours()
        opt = train.build_optimizer(m, base_lr=0.1)
        assert isinstance(opt, train.FusedSGD)
        ga = GradAllReduce(m, defer_scale_to=opt)
        base = ga.flat.data_ptr()
        for _ in range(2):
            out = m(x)
            loss = torch.nn.functional.cross_entropy(out, labels)
            opt.zero_grad(set_to_none=True)
            loss.backward()
            torch.cuda.synchronize()
            for (n, p), off in zip(ga.named, ga.offsets):
                assert p.grad is not None and p.grad.data_ptr() == base + 4 * off, n
            ga()
            assert ga.copied == 0
            opt.step()
        torch.cuda.synchronize()
        for (n, a), (_, b) in zip(m.named_parameters(), m_ref.named_parameters()):
            assert torch.equal(a, b), n
        ga.close()
    finally:
        dist.destroy_process_group()


def test_fc_gradients_in_slots_match_nn_linear():
    """head.linear (the classifier with its gradients written into bucket slots) computes
    the same calls as torch's addmm backward: bit-identical gradients."""
    from shiftgcn import head, ops
    g = torch.Generator().manual_seed(3)
    fc = torch.nn.Linear(256, 60).to(DEV)
    fc2 = torch.nn.Linear(256, 60).to(DEV)
    fc2.load_state_dict(fc.state_dict())
    x = torch.randn(64, 256, generator=g).to(DEV)
    gy = torch.randn(64, 60, generator=g).to(DEV)
    flat = torch.zeros(fc.weight.numel() + fc.bias.numel(), device=DEV)
    ops.register_grad_slots([("w", fc.weight), ("b", fc.bias)], flat)
    try:
        x1 = x.clone().requires_grad_(True)
        x2 = x.clone().requires_grad_(True)
        head.linear(fc, x1).backward(gy)
        fc2(x2).backward(gy)
        torch.cuda.synchronize()
        assert fc.weight.grad.data_ptr() == flat.data_ptr()
        assert torch.equal(fc.weight.grad, fc2.weight.grad)
        assert torch.equal(fc.bias.grad, fc2.bias.grad)
        assert torch.equal(x1.grad, x2.grad)
    finally:
        ops.unregister_grad_slots([fc.weight, fc.bias])
