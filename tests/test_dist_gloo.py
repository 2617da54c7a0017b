"""Data-parallel semantics on CPU with gloo, world_size 2 (two processes).

Checks the nn.DataParallel-equivalent reduction rule of shiftgcn.dist.GradAllReduce
(SURVEY §8e): ordinary parameter gradients are MEANED over ranks (== DataParallel's sum
of replica grads of the global-mean loss), shift-position gradients (xpos/ypos, already
sign-normalised per replica) are SUMMED; BN running stats are taken from rank 0.
"""
import os
import socket

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
        q.put((rank, m.lin.weight.grad.clone(), m.lin.bias.grad.clone(),
               m.shift.ypos.grad.clone(), m.bn.running_mean.clone(), m.lin.weight.detach().clone()))
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
