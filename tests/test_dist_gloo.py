"""Data-parallel semantics on CPU with gloo, world_size 2 (two processes).

Checks the nn.DataParallel-equivalent reduction rule of shiftgcn.dist.GradAllReduce
(SURVEY §8e): ordinary parameter gradients are MEANED over ranks (== DataParallel's sum
of replica grads of the global-mean loss), shift-position gradients (xpos/ypos, already
sign-normalised per replica) are SUMMED; BN running stats are taken from rank 0.

``test_real_model_*`` run the REAL parameter set (the CPU oracle of ``model/shift_gcn.py``:
693,107 trainable parameters incl. 20x2 shift-position vectors, 50 BatchNorms, the int64
index parameters) through GradAllReduce on two half-batches and compare with the
single-process DataParallel restatement (``oracle/dp_oracle.py``, main.py:294-299).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG_ROOT


class Toy(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.lin = torch.nn.Linear(3, 2)
        self.shift = torch.nn.Module()
        self.shift.xpos = torch.nn.Parameter(torch.zeros(4))
        self.shift.ypos = torch.nn.Parameter(torch.zeros(4))
        self.bn = torch.nn.BatchNorm1d(2)
        self.idx = torch.nn.Parameter(torch.arange(5), requires_grad=False)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, PKG_ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from shiftgcn.dist import GradAllReduce, broadcast_buffers, broadcast_parameters
        torch.manual_seed(100 + rank)
        m = Toy()
        broadcast_parameters(m)
        m.lin.weight.grad = torch.full_like(m.lin.weight, float(rank + 1))
        m.lin.bias.grad = torch.full_like(m.lin.bias, 10.0 * (rank + 1))
        m.shift.xpos.grad = torch.zeros(4)
        m.shift.ypos.grad = (torch.tensor([0.01, -0.01, 0.01, 0.0001]) if rank == 0 else
                             torch.tensor([0.01, 0.01, -0.01, 0.0001]))
        m.bn.running_mean.fill_(float(rank + 7))
        GradAllReduce(m)()
        broadcast_buffers(m)
        # numpy, not tensors: a tensor in a queue is shared through a socket owned by this
        # process, which may already have exited when the parent unpickles it
        q.put((rank,) + tuple(t.detach().numpy().copy() for t in (
            m.lin.weight.grad, m.lin.bias.grad, m.shift.ypos.grad, m.bn.running_mean,
            m.lin.weight)))
    finally:
        dist.destroy_process_group()


def test_grad_allreduce_dataparallel_rule_gloo_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda r: r[0])
    res = [(r[0],) + tuple(torch.from_numpy(a) for a in r[1:]) for r in res]
    for rank, w, b, y, rm, wt in res:
        assert torch.allclose(w, torch.full_like(w, 1.5))            # mean of 1 and 2
        assert torch.allclose(b, torch.full_like(b, 15.0))           # mean of 10 and 20
        # ypos: SUM of the per-rank sign-normalised grads (DataParallel reduce-add)
        assert torch.allclose(y, torch.tensor([0.02, 0.0, 0.0, 0.0002]))
        assert torch.allclose(rm, torch.full_like(rm, 7.0))          # rank 0's running stats
    assert torch.equal(res[0][5], res[1][5])                          # params broadcast


@pytest.mark.parametrize("rule", ["sum", "mean"])
def test_scale_vector_single_process(rule):
    """The per-element scale vector: 1/world for ordinary params, 1 (sum) for shifts."""
    import sys
    sys.path.insert(0, PKG_ROOT)
    from shiftgcn.dist import is_shift_position
    assert is_shift_position("l1.tcn1.shift_in.ypos") and is_shift_position("a.xpos")
    assert not is_shift_position("l1.gcn1.Linear_weight")


# --------------------------------------------------------------------------------------
# the real model (oracle restatement of model/shift_gcn.py) through GradAllReduce
# --------------------------------------------------------------------------------------
REAL = dict(N=4, T=24, V=25, M=2, num_class=60, seed=123)


def _real_inputs():
    import formula
    x = formula.tensor((REAL["N"], 3, REAL["T"], REAL["V"], REAL["M"]), 77, 1.0)
    labels = torch.arange(REAL["N"]) * 7 % REAL["num_class"]
    return x, labels


def _real_model():
    import formula
    from oracle import model_oracle as mo
    m = mo.Model(num_class=REAL["num_class"], num_point=REAL["V"], num_person=REAL["M"])
    formula.fill_state(m, seed=REAL["seed"])
    return m.train()


def _real_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, PKG_ROOT)
    from conftest import GOLDEN, REPO
    for p in (REPO, GOLDEN):
        sys.path.insert(0, p)
    torch.set_num_threads(1)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from shiftgcn.dist import GradAllReduce, broadcast_buffers, broadcast_parameters
        m = _real_model()
        broadcast_parameters(m)
        x, labels = _real_inputs()
        n = x.shape[0] // world
        xs, ls = x[rank * n:(rank + 1) * n], labels[rank * n:(rank + 1) * n]
        loss = torch.nn.functional.cross_entropy(m(xs), ls)    # local-mean loss per rank
        m.zero_grad(set_to_none=True)
        loss.backward()
        GradAllReduce(m)()
        broadcast_buffers(m)
        # numpy across the queue (tensor storages would be fd-shared with an exiting process)
        q.put((rank, {k: p.grad.numpy().copy() for k, p in m.named_parameters()
                      if p.requires_grad},
               {k: b.numpy().copy() for k, b in m.named_buffers()}))
    finally:
        dist.destroy_process_group()


def _spawn(target, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(res, key=lambda r: r[0])


def test_real_model_grad_allreduce_equals_dataparallel_gloo_world2():
    """Two gloo ranks x half batch == nn.DataParallel(k=2) on the whole batch, bit for bit:
    the local-mean CE gradient is exactly 2x the replica's global-mean one (a power of two),
    so sum-then-halve reproduces DataParallel's replica sum exactly; xpos/ypos are the SUM
    of the per-rank +-0.01; every rank ends with replica 0's BN running statistics."""
    from oracle.dp_oracle import dataparallel_grads
    res = _spawn(_real_worker)
    prev = torch.get_num_threads()
    torch.set_num_threads(1)
    try:
        ref = _real_model()
        x, labels = _real_inputs()
        _, _, g_dp = dataparallel_grads(ref, x, labels, 2)
    finally:
        torch.set_num_threads(prev)
    n_shift = 0
    for rank, grads, bufs in res:
        assert set(grads) == set(g_dp)
        for k, g in grads.items():
            gd = g_dp[k].numpy()
            assert np.array_equal(g, gd), (rank, k, float(np.abs(g - gd).max()))
            if k.endswith("ypos"):
                # the sum of two sign-normalised replica grads: 0 or +-0.02
                vals = set(np.round(g / 0.01).astype(int).tolist())
                assert vals <= {-2, 0, 2}, (k, vals)
                n_shift += 1
        for k, b in ref.named_buffers():
            assert np.array_equal(bufs[k], b.numpy()), (rank, k)
    assert n_shift == 2 * 20   # 2 ranks x 10 units x (shift_in, shift_out)


def _defer_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, PKG_ROOT)
    torch.set_num_threads(1)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from shiftgcn.dist import GradAllReduce, broadcast_parameters
        from shiftgcn.train import FusedSGD
        out = {}
        for defer in (False, True):
            torch.manual_seed(5)
            m = Toy()
            broadcast_parameters(m)
            opt = (FusedSGD if defer else torch.optim.SGD)(
                [p for p in m.parameters() if p.requires_grad], lr=0.1, momentum=0.9,
                nesterov=True, weight_decay=1e-4)
            ga = GradAllReduce(m, defer_scale_to=opt if defer else None)
            for step in range(2):
                g = torch.Generator().manual_seed(50 * step + rank)
                for p in m.parameters():
                    if p.requires_grad:
                        p.grad = torch.randn(p.shape, generator=g)
                ga()
                # every .grad is its bucket slot after the call
                base = ga.flat.data_ptr()
                assert all(p.grad.data_ptr() == base + 4 * off
                           for (_, p), off in zip(ga.named, ga.offsets))
                opt.step()
            ga.close()
            out[defer] = {n: p.detach().numpy().copy() for n, p in m.named_parameters()
                          if p.requires_grad}
            out[(defer, "grad")] = {n: p.grad.numpy().copy() for n, p in m.named_parameters()
                                    if p.requires_grad}
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_deferred_scale_matches_multiply_then_step_gloo_world2():
    """GradAllReduce(defer_scale_to=FusedSGD): the DataParallel 1/world applied inside the
    optimizer step (here the host fallback: one multiply, then torch's update) leaves the
    same parameters AND the same .grad as the scale applied by GradAllReduce itself."""
    res = _spawn(_defer_worker)
    for rank, out in res:
        for key in (False, (False, "grad")):
            other = True if key is False else (True, "grad")
            for n, v in out[key].items():
                assert np.array_equal(v, out[other][n]), (rank, key, n)


def _clip_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, PKG_ROOT)
    torch.set_num_threads(1)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from shiftgcn.dist import GradAllReduce, broadcast_parameters
        from shiftgcn.train import FusedSGD
        out = {}
        for defer in (False, True):
            torch.manual_seed(5)
            m = Toy()
            broadcast_parameters(m)
            opt = (FusedSGD if defer else torch.optim.SGD)(
                [p for p in m.parameters() if p.requires_grad], lr=0.1, momentum=0.9,
                nesterov=True, weight_decay=1e-4)
            ga = GradAllReduce(m, defer_scale_to=opt if defer else None)
            g = torch.Generator().manual_seed(7 + rank)
            for p in m.parameters():
                if p.requires_grad:
                    p.grad = 3.0 * torch.randn(p.shape, generator=g)
            ga()
            out[(defer, "norm")] = float(ga.clip_grad_norm_(0.5))
            opt.step()
            ga.close()
            out[defer] = {n: p.detach().numpy().copy() for n, p in m.named_parameters()
                          if p.requires_grad}
        # reference: reduce by hand, clip with torch, step
        torch.manual_seed(5)
        m = Toy()
        broadcast_parameters(m)
        opt = torch.optim.SGD([p for p in m.parameters() if p.requires_grad], lr=0.1,
                              momentum=0.9, nesterov=True, weight_decay=1e-4)
        g = torch.Generator().manual_seed(7 + rank)
        for n, p in m.named_parameters():
            if p.requires_grad:
                p.grad = 3.0 * torch.randn(p.shape, generator=g)
                dist.all_reduce(p.grad)
                if not (n.endswith(".xpos") or n.endswith(".ypos")):
                    p.grad.mul_(1.0 / world)
        out["torch_norm"] = float(torch.nn.utils.clip_grad_norm_(
            [p for p in m.parameters() if p.requires_grad], 0.5))
        opt.step()
        out["torch"] = {n: p.detach().numpy().copy() for n, p in m.named_parameters()
                        if p.requires_grad}
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_clip_grad_norm_in_both_scale_forms_gloo_world2():
    """with the deferred scale, .grad holds the rank SUM until step();
    GradAllReduce.clip_grad_norm_ clips the REDUCED gradients in both forms, matching
    torch.nn.utils.clip_grad_norm_ over the reduced .grad followed by torch's SGD."""
    res = _spawn(_clip_worker)
    for rank, out in res:
        for defer in (False, True):
            assert abs(out[(defer, "norm")] - out["torch_norm"]) <= 1e-5 * out["torch_norm"]
            for n, v in out[defer].items():
                np.testing.assert_allclose(v, out["torch"][n], rtol=1e-6, atol=1e-7,
                                           err_msg=f"{rank} {defer} {n}")
