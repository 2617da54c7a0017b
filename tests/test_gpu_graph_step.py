"""GPU: the whole training step (forward, CrossEntropy, backward with the weight gradients
on the side stream, FusedSGD) captured in a hipGraph (`bench.py --graph 1`) and replayed
gives the same parameters, momentum buffers and BatchNorm statistics, bit for bit, as the
same number of eager steps. Every kernel is deterministic, so a replay that read a stale
optimizer table or raced the side stream would show up as a mismatch."""
import copy

import pytest
import torch

import formula

pytestmark = pytest.mark.gpu


def _setup(dev):
    import shiftgcn
    from shiftgcn import train
    m = shiftgcn.Model(num_class=10, num_point=25, num_person=2, graph="graph.ntu_rgb_d.Graph")
    formula.fill_state(m, seed=9)
    m = m.to(dev).train()
    x = formula.tensor((4, 3, 64, 25, 2), 77, 1.0).to(dev)
    y = torch.tensor([1, 3, 5, 7], device=dev)
    return m, x, y, train


def test_graph_replayed_training_step_matches_eager():
    dev = torch.device("cuda:0")
    m, x, y, train = _setup(dev)
    m2 = copy.deepcopy(m)
    opt = train.build_optimizer(m, base_lr=0.1)
    opt2 = train.build_optimizer(m2, base_lr=0.1)
    assert isinstance(opt2, train.FusedSGD)

    # eager: 6 steps
    for _ in range(6):
        train.train_step(m, opt, x, y)
    # graph: 2 eager warm-up steps, one on a side stream (as bench.py does), capture, 3 replays
    for _ in range(2):
        train.train_step(m2, opt2, x, y)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        train.train_step(m2, opt2, x, y)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        train.train_step(m2, opt2, x, y)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()

    for (n, a), (_, b) in zip(m.named_parameters(), m2.named_parameters()):
        assert torch.equal(a, b), n
    for (n, a), (_, b) in zip(m.named_buffers(), m2.named_buffers()):
        assert torch.equal(a, b), n
    for p, p2 in zip(m.parameters(), m2.parameters()):
        if p.requires_grad:
            assert torch.equal(opt.state[p]["momentum_buffer"], opt2.state[p2]["momentum_buffer"])
