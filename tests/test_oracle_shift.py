"""Pin the temporal-shift oracle (CPU; no GPU needed).

The reference CUDA extension cannot run here, so the restatement is pinned by:
(1) a second, scalar-loop restatement (bit-exact agreement), (2) hand-derived known
answers, (3) the exact-adjoint property of the bottom backward (float64), and (4) the
fixtures produced through the reference's own ``ShiftFunction`` glue (``shift.py``).
"""
import numpy as np
import pytest
import torch

from oracle import shift_loops as sl
from oracle import shift_oracle as so
from gen_fixtures import SHIFT_CASES, shift_case_inputs

F32 = np.float32


@pytest.mark.parametrize("stride,H", [(1, 7), (1, 8), (2, 7), (2, 8)])
def test_vectorised_equals_scalar_loops(stride, H):
    rng = np.random.default_rng(stride * 10 + H)
    B, C, W = 2, 7, 5
    x = rng.standard_normal((B, C, H, W)).astype(F32)
    xp = np.array([1e-8, -1e-8, 0, 1.3, -2.7, 0.5, 7.0], F32)
    yp = so.effective_ypos(np.array([-3.2, 0.0, 2.0, 1.7, -0.4, 9.0, -8.5], F32), stride)
    out = so.shift_forward(x, xp, yp, stride)
    assert np.array_equal(out, sl.forward(x, xp, yp, stride))
    g = rng.standard_normal(out.shape).astype(F32)
    assert np.array_equal(so.shift_bottom_backward(g, xp, yp, H, stride),
                          sl.bottom_backward(g, xp, yp, H, stride))
    a = so.shift_position_backward(x, g, xp, yp, stride)
    b = sl.position_backward(x, g, xp, yp, stride)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_integer_shift_is_translation():
    """Known answer: integer ypos k, xpos 0 -> out[h] = in[h*s + k] (zero outside)."""
    rng = np.random.default_rng(1)
    x = rng.standard_normal((1, 3, 10, 4)).astype(F32)
    yp = np.array([2.0, -3.0, 0.0], F32)
    xp = np.zeros(3, F32)
    out = so.shift_forward(x, xp, yp, 1)
    for c, k in enumerate([2, -3, 0]):
        for h in range(10):
            hs = h + k
            ref = x[0, c, hs] if 0 <= hs < 10 else np.zeros(4, F32)
            assert np.array_equal(out[0, c, h], ref)
    # xpos = +1 moves along the joint axis, the last joint reads zero padding
    out = so.shift_forward(x, np.ones(3, F32), np.zeros(3, F32), 1)
    assert np.array_equal(out[..., :3], x[..., 1:]) and not out[..., 3].any()


def test_demo_case_ones_stride2():
    """The reference demo (``model/Temporal_shift/demo.py``): Shift(5, stride=2) on
    ones(1,5,8,4). With the effective shift y = ypos + 0.5 in [0,1) the interior taps are
    all ones, so out == 1 except where the second tap row (2h+1) ... stays in range: for
    stride 2 and H=8 every tap row 2h+{0,1} <= 7 is in range -> out == 1 exactly."""
    x = np.ones((1, 5, 8, 4), F32)
    ypos = np.array([-0.5, -0.25, 0.0, 0.2, 0.49], F32)
    out = so.shift_forward(x, np.zeros(5, F32), so.effective_ypos(ypos, 2), 2)
    assert out.shape == (1, 5, 4, 4)
    assert np.array_equal(out, np.ones_like(out))
    g = np.ones_like(out)
    gin, gx, gy = so.shift_backward(g, x, np.zeros(5, F32), so.effective_ypos(ypos, 2), 2)
    # constant input -> all position gradients vanish -> constraint's dr==0 branch
    assert np.array_equal(gy, np.full(5, F32(0.0001))) and np.array_equal(gx, np.zeros(5, F32))
    # every input row is hit by total weight 1 (each output row splits weight 1 over 2 rows)
    assert np.allclose(gin.sum(), out.size)


@pytest.mark.parametrize("stride", [1, 2])
def test_bottom_backward_is_adjoint(stride):
    rng = np.random.default_rng(5 + stride)
    x = rng.standard_normal((2, 6, 12, 5)).astype(F32)
    xp = np.array([0.0, 1e-8, -1e-8, 0.7, -1.2, 2.0], F32)
    yp = so.effective_ypos(np.array([0.0, 1.0, -2.0, 0.3, -0.6, 5.5], F32), stride)
    y = so.shift_forward(x, xp, yp, stride)
    g = rng.standard_normal(y.shape).astype(F32)
    gin = so.shift_bottom_backward(g, xp, yp, 12, stride)
    lhs = float((y.astype(np.float64) * g).sum())
    rhs = float((x.astype(np.float64) * gin).sum())
    assert abs(lhs - rhs) < 1e-5 * max(1.0, abs(lhs))


def test_constraint_edges():
    gx, gy = so.apply_shift_constraint(np.array([3.0, -2.0, 5.0, 1e-30], F32),
                                       np.array([2.0, -7.0, 0.0, 1e-30], F32))
    assert gy[0] == F32(0.01) and gy[1] == -F32(0.01)
    assert gy[2] == F32(0.0001) and gx[2] == 0.0
    # 1e-30**2 underflows to 0 in float32 -> the dr == 0 branch
    assert gy[3] == F32(0.0001)
    assert np.all(gx[:2] == 0.0)
    assert np.signbit(gx[1]) and not np.signbit(gx[0])   # (dx/dr)*0.0 keeps the sign


@pytest.mark.parametrize("case", SHIFT_CASES, ids=[c[0] for c in SHIFT_CASES])
def test_oracle_matches_reference_glue_fixture(golden, case):
    """The fixtures ran the reference ``ShiftFunction`` (+0.5 for stride 2, saved ypos)."""
    fx = golden("shift_fixtures.npz")
    name, B, C, H, W, stride = case
    x, g, xpos, ypos = (t.numpy() for t in shift_case_inputs(*case))
    ye = so.effective_ypos(ypos, stride)
    assert np.array_equal(so.shift_forward(x, xpos, ye, stride), fx[f"shift_{name}_out"])
    gin, gx, gy = so.shift_backward(g, x, xpos, ye, stride)
    assert np.array_equal(gin, fx[f"shift_{name}_gin"])
    assert np.array_equal(gx, fx[f"shift_{name}_gx"])
    assert np.array_equal(gy, fx[f"shift_{name}_gy"])


def test_effective_ypos_is_torch_fp32_add():
    y = np.array([0.1, -0.3, 1e-8, 2.5, -0.5], F32)
    assert np.array_equal(so.effective_ypos(y, 2), (torch.from_numpy(y) + 0.5).numpy())


@pytest.mark.parametrize("stride", [1, 2])
def test_fma_contracted_variant_is_within_one_rounding(stride):
    """The FMA-contracted restatement (nvcc --fmad=true of .cu:73, .cu:343-344) differs from
    the uncontracted one only by rounding: forward / input gradient within 1e-6 relative to
    the tensor scale (well inside the 1e-5 bar), identical constrained position grads up
    to sign flips of near-zero plane sums."""
    rng = np.random.default_rng(11 + stride)
    B, C, H, W = 2, 8, 40, 25
    x = rng.standard_normal((B, C, H, W)).astype(np.float32)
    xpos = rng.uniform(-1e-8, 1e-8, C).astype(np.float32)
    ypos = so.effective_ypos(rng.uniform(-3, 3, C).astype(np.float32), stride)
    g = rng.standard_normal((B, C, H // stride, W)).astype(np.float32)
    a = so.shift_forward(x, xpos, ypos, stride)
    b = so.shift_forward(x, xpos, ypos, stride, contract=True)
    assert np.abs(a - b).max() <= 1e-6 * np.abs(a).max()
    ga, gxa, gya = so.shift_backward(g, x, xpos, ypos, stride)
    gb, gxb, gyb = so.shift_backward(g, x, xpos, ypos, stride, contract=True)
    assert np.abs(ga - gb).max() <= 1e-6 * np.abs(ga).max()
    assert (gya != gyb).sum() <= 1 and (gxa != gxb).sum() <= 1
    # integer shifts (dx = dy = 0): contraction cannot change a pure translation
    yi = np.round(ypos).astype(np.float32)
    assert np.array_equal(so.shift_forward(x, np.zeros_like(xpos), yi, 1),
                          so.shift_forward(x, np.zeros_like(xpos), yi, 1, contract=True))


@pytest.mark.parametrize("stride", [1, 2])
def test_torch_restatement_matches_numpy_oracle(stride):
    """oracle/torch_shift.py (the on-device eager reference of the full-size parity tests)
    agrees with the numpy oracle on the CPU."""
    from oracle import torch_shift as ts
    rng = np.random.default_rng(5 + stride)
    B, C, H, W = 2, 8, 30, 25
    x = rng.standard_normal((B, C, H, W)).astype(np.float32)
    xpos = rng.uniform(-1e-8, 1e-8, C).astype(np.float32)
    xpos[1] = 1.5
    ypos = so.effective_ypos(rng.uniform(-3, 3, C).astype(np.float32), stride)
    ypos[2] = float(H + 2)
    g = rng.standard_normal((B, C, H // stride, W)).astype(np.float32)
    out = ts.shift_forward(torch.from_numpy(x), torch.from_numpy(xpos), torch.from_numpy(ypos),
                           stride).numpy()
    ref = so.shift_forward(x, xpos, ypos, stride)
    assert np.abs(out - ref).max() <= 1e-6 * np.abs(ref).max()
    gin, gx, gy = ts.shift_backward(torch.from_numpy(g), torch.from_numpy(x),
                                    torch.from_numpy(xpos), torch.from_numpy(ypos), stride)
    rgin, rgx, rgy = so.shift_backward(g, x, xpos, ypos, stride)
    assert np.abs(gin.numpy() - rgin).max() <= 1e-6 * np.abs(rgin).max()
    assert (gy.numpy() != rgy).sum() <= 1 and (gx.numpy() != rgx).sum() <= 1
