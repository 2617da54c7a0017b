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


@pytest.fixture(autouse=True)
def _fresh_cache_state(monkeypatch):
    # capturing a training step switches the eval caches off for the process (ops.
    # mark_captured_writes); keep that to this module's tests
    from shiftgcn import ops
    monkeypatch.setattr(ops, "_CAPTURED_WRITES", False)


def _capture(m2, opt2, x, y, train, warm=2):
    """``warm`` eager steps, one on a side stream (as bench.py does), then the captured
    step (not run by the capture)."""
    for _ in range(warm):
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
    return g


def _same_state(m, m2, opt, opt2):
    for (n, a), (_, b) in zip(m.named_parameters(), m2.named_parameters()):
        assert torch.equal(a, b), n
    for (n, a), (_, b) in zip(m.named_buffers(), m2.named_buffers()):
        assert torch.equal(a, b), n
    for p, p2 in zip(m.parameters(), m2.parameters()):
        if p.requires_grad:
            assert torch.equal(opt.state[p]["momentum_buffer"], opt2.state[p2]["momentum_buffer"])


def test_graph_replay_follows_learning_rate_changes():
    """``adjust_learning_rate`` (main.py:342-353) between replays of a
    captured step: the replays use the new lr (FusedSGD's device-resident hyper-parameters),
    bit for bit as eager steps with the same schedule."""
    dev = torch.device("cuda:0")
    m, x, y, train = _setup(dev)
    m2 = copy.deepcopy(m)
    opt = train.build_optimizer(m, base_lr=0.1)
    opt2 = train.build_optimizer(m2, base_lr=0.1)
    epochs = (0, 60, 80)
    for _ in range(4):
        train.train_step(m, opt, x, y)
    for e in epochs[1:]:
        train.adjust_learning_rate(opt, e)
        train.train_step(m, opt, x, y)
    g = _capture(m2, opt2, x, y, train)
    for e in epochs:
        train.adjust_learning_rate(opt2, e)
        g.replay()
    torch.cuda.synchronize()
    assert [h[1] for h in opt2._hyper_host] == [pytest.approx(1e-3)] * len(opt2.param_groups)
    _same_state(m, m2, opt, opt2)
    # one more step at the last learning rate
    g.replay()
    train.train_step(m, opt, x, y)
    torch.cuda.synchronize()
    _same_state(m, m2, opt, opt2)


def test_eval_after_graph_replays_reads_current_weights():
    """capture, replay, eval, replay, eval — the second eval must use
    the weights and running statistics of the later replays (no version-keyed cache hit),
    equal to eager steps with evals at the same points."""
    from shiftgcn import ops
    dev = torch.device("cuda:0")
    m, x, y, train = _setup(dev)
    m2 = copy.deepcopy(m)
    opt = train.build_optimizer(m, base_lr=0.1)
    opt2 = train.build_optimizer(m2, base_lr=0.1)
    xe = formula.tensor((2, 3, 64, 25, 2), 78, 1.0).to(dev)

    def ev(model):
        model.eval()
        with torch.no_grad():
            out = model(xe).clone()
        model.train()
        return out

    outs = []
    for k in range(7):
        train.train_step(m, opt, x, y)
        if k in (4, 6):
            outs.append(ev(m))
    g = _capture(m2, opt2, x, y, train)
    assert ops._CAPTURED_WRITES
    got = []
    for _ in range(2):
        g.replay()
    got.append(ev(m2))
    for _ in range(2):
        g.replay()
    got.append(ev(m2))
    torch.cuda.synchronize()
    assert not torch.equal(outs[0], outs[1])
    for a, b in zip(outs, got):
        assert torch.equal(a, b)


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
