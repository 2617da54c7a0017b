"""Training BatchNorm finalizes run in the tail of the launch that makes their partials
(round 4, sgcn_bn_fin): the workgroup completing a channel merges the channel's batch
partials in sgcn_bn_finalize's order, so every statistic must be BIT-identical to the
separate finalize launch — mean/invstd/scale/shift, the running statistics and
num_batches_tracked — for the BatchNorm2d (model/shift_gcn.py:38,55-56,85) and the
per-joint BatchNorm1d(V*C) of Shift_gcn (:99,137), and the counters must be left zero so
repeated launches stay correct."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _bn(F, seed, one_d=False):
    g = torch.Generator().manual_seed(seed)
    bn = (torch.nn.BatchNorm1d(F) if one_d else torch.nn.BatchNorm2d(F)).to(DEV)
    with torch.no_grad():
        bn.weight.copy_(torch.rand(F, generator=g) + 0.5)
        bn.bias.copy_(torch.randn(F, generator=g))
        bn.running_mean.copy_(torch.randn(F, generator=g))
        bn.running_var.copy_(torch.rand(F, generator=g) + 0.5)
    return bn


def _stats(st, bn):
    return (st.mean.clone(), st.invstd.clone(), st.scale.clone(), st.shift.clone(),
            bn.running_mean.clone(), bn.running_var.clone(), int(bn.num_batches_tracked))


def _coefs(st):
    return (st.mean.clone(), st.invstd.clone(), st.scale.clone(), st.shift.clone())


@pytest.mark.parametrize("B,C,T,V", [(1, 4, 30, 25), (3, 8, 12, 70), (9, 16, 30, 25),
                                     (128, 64, 300, 25), (33, 256, 75, 25), (5, 32, 75, 33),
                                     (4, 8, 1000, 25)])
@pytest.mark.parametrize("per_joint", [0, 3])
def test_moments_tail_finalize_bit_identical(B, C, T, V, per_joint):
    from shiftgcn import ops
    g = torch.Generator().manual_seed(B * 7 + C + T + V + per_joint)
    x = (torch.randn(B, C, T, V, generator=g) * 1.7 + 0.4).to(DEV)
    F = C * (V if per_joint else 1)
    n_part = T if per_joint else T * V
    bn_a, bn_b = _bn(F, 3, per_joint != 0), _bn(F, 3, per_joint != 0)
    ref = ops.bn_finalize(ops.moments(x, per_joint), B, F, n_part, bn_a,
                          perm_V=V if per_joint else 0)
    want = _stats(ref, bn_a)
    for rep in range(3):   # the counters come back to zero: repeated launches agree
        st = ops.moments_bn(x, per_joint, bn_b)
        torch.cuda.synchronize()
        got = _stats(st, bn_b)
        for a, b in zip(want[:4], got[:4]):
            assert torch.equal(a, b)
        if rep == 0:
            assert torch.equal(want[4], got[4]) and torch.equal(want[5], got[5])
            assert got[6] == 1
    assert int(bn_b.num_batches_tracked) == 3
    cnt = ops._fin_count(x.device, C)
    assert int(cnt.abs().sum()) == 0


def test_moments_tail_finalize_untracked_and_affine_free():
    from shiftgcn import ops
    x = torch.randn(6, 12, 20, 25, device=DEV)
    bn_a = torch.nn.BatchNorm2d(12, affine=False, track_running_stats=False).to(DEV)
    bn_b = torch.nn.BatchNorm2d(12, affine=False, track_running_stats=False).to(DEV)
    ref = ops.bn_finalize(ops.moments(x, 0), 6, 12, 500, bn_a)
    st = ops.moments_bn(x, 0, bn_b)
    for a, b in zip(_coefs(ref), _coefs(st)):
        assert torch.equal(a, b)
    # against torch's own BatchNorm2d in train()
    y = torch.nn.functional.batch_norm(x, None, None, training=True, eps=bn_b.eps)
    mine = x * st.scale.view(1, -1, 1, 1) + st.shift.view(1, -1, 1, 1)
    assert torch.allclose(mine, y, atol=1e-5, rtol=1e-5)


def test_moments_tail_finalize_side_stream_counters():
    """Two streams running tail finalizes concurrently use separate counters."""
    from shiftgcn import ops
    x = torch.randn(16, 32, 60, 25, device=DEV)
    y = torch.randn(16, 32, 60, 25, device=DEV) * 3
    bn_x, bn_y = _bn(32, 1), _bn(32, 2)
    rx = ops.bn_finalize(ops.moments(x, 0), 16, 32, 1500, _bn(32, 1))
    ry = ops.bn_finalize(ops.moments(y, 0), 16, 32, 1500, _bn(32, 2))
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    for _ in range(4):
        sx = ops.moments_bn(x, 0, bn_x)
        with torch.cuda.stream(side):
            sy = ops.moments_bn(y, 0, bn_y)
    torch.cuda.synchronize()
    assert torch.equal(sx.scale, rx.scale) and torch.equal(sx.shift, rx.shift)
    assert torch.equal(sy.scale, ry.scale) and torch.equal(sy.shift, ry.shift)
