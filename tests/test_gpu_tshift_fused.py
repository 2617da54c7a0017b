"""Shift_tcn's shift_in fused into its temporal_linear (north_star: "the learnable
fractional temporal shift ... fused with its trailing pointwise 1x1 conv"; reference
model/shift_gcn.py:66-69, shift_cuda_kernel.cu:11-76).

* forward: ``sgcn_pw_fwd_tshift`` == ``sgcn_tshift_fwd`` (bn affine on the taps) followed
  by ``sgcn_pw_fwd``, bit for bit (same tap arithmetic, same K order), including planes
  whose position count is not a tile multiple, |ypos| > 1, x shifts of a whole joint, V=33;
* the side output is the shifted operand, element for element (the weight gradient's
  operand, read by ``sgcn_pw_dw``);
* the fused form and the two-launch form give the same unit parity vs the oracle;
* in a training step there is no separate shift_in launch for the units at or above the
  channel threshold: the other temporal-shift forward launches are the 10 shift_outs
  (whose output feeds bn2's statistics).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"

CASES = [
    # (B, K, M, T, V)
    (3, 64, 64, 20, 25),
    (2, 128, 128, 17, 25),      # P not a multiple of the 256-position tile
    (2, 256, 256, 9, 25),
    (3, 64, 64, 11, 33),
    (1, 128, 256, 7, 25),
]


def _inputs(B, K, M, T, V, seed):
    g = torch.Generator().manual_seed(seed)
    h = torch.randn(B, K, T, V, generator=g).to(DEV)
    w = (torch.randn(M, K, generator=g) / K ** 0.5).to(DEV)
    bias = torch.randn(M, generator=g).to(DEV)
    xpos = ((torch.rand(K, generator=g) - 0.5) * 2e-8)
    ypos = (torch.rand(K, generator=g) - 0.5) * 6          # |y| up to 3 (> 1 tap row)
    xpos[0], ypos[0] = 1.0, 0.0                            # a whole-joint x shift
    xpos[1] = -1.5
    ypos[2] = float(T + 1)                                 # shifted out of the plane
    scale = (torch.rand(K, generator=g) + 0.5).to(DEV)
    shift = torch.randn(K, generator=g).to(DEV)
    return h, w, bias, xpos.to(DEV), ypos.to(DEV), scale, shift


class _St:
    def __init__(self, scale, shift):
        self.scale, self.shift = scale, shift


@pytest.mark.parametrize("case", CASES, ids=["x".join(map(str, c)) for c in CASES])
def test_fused_forward_bit_identical_to_two_launch(case):
    from shiftgcn import ops
    from shiftgcn.ops import PlaneView as PV
    B, K, M, T, V = case
    h, w, bias, xpos, ypos, scale, shift = _inputs(*case, seed=sum(case))
    As = ops.tshift_fwd(h, xpos, ypos, 1, scale=scale, shift=shift)
    r1 = torch.empty(B, M, T, V, device=DEV)
    ops.pw_fwd(w, False, bias, PV(As), PV(r1), M, K, T, V, relu=True)
    r2 = torch.empty(B, M, T, V, device=DEV)
    ops.pw_fwd_tshift(w, bias, PV(h), xpos, ypos, _St(scale, shift), PV(r2), M, K, T, V,
                      relu=True)
    r3 = torch.empty(B, M, T, V, device=DEV)
    xs = torch.full_like(h, float("nan"))
    ops.pw_fwd_tshift(w, bias, PV(h), xpos, ypos, _St(scale, shift), PV(r3), M, K, T, V,
                      relu=True, x_shifted=xs)
    torch.cuda.synchronize()
    assert torch.equal(r1, r2) and torch.equal(r1, r3)
    assert torch.equal(xs, As)        # the side output is the shifted operand, every element


@pytest.mark.parametrize("min_c", [0, 1024])
def test_unit_matches_oracle_fused_and_two_launch(monkeypatch, min_c):
    """The fused shift_in contraction (threshold 0: the C = 128 unit below takes it) and the
    two-launch form (threshold above every width) give the same unit parity."""
    import formula
    import shiftgcn
    from oracle import model_oracle as mo
    from shiftgcn import fused
    from test_gpu_blocks import _compare
    monkeypatch.setattr(fused, "TSHIFT_FUSION_MIN_C", min_c)
    ref = mo.TCN_GCN_unit(64, 128, None, stride=2, num_point=25)
    formula.fill_state(ref, seed=min_c + 17)
    ours = shiftgcn.TCN_GCN_unit(64, 128, None, stride=2, num_point=25).to(DEV)
    ours.load_state_dict(ref.state_dict())
    ref.train()
    ours.train()
    x = formula.tensor((3, 64, 18, 25), 50 + min_c, 1.0)
    g = formula.tensor((3, 128, 9, 25), 60 + min_c, 1.0)
    xr = x.clone().requires_grad_(True)
    yr = ref(xr)
    yr.backward(g)
    xo = x.to(DEV).requires_grad_(True)
    yo = ours(xo)
    yo.backward(g.to(DEV))
    torch.cuda.synchronize()
    _compare(ref, ours, xr, yr, xo, yo, f"min_c{min_c}")


@pytest.mark.parametrize("min_c", [0, None])
def test_training_step_has_no_shift_in_launch(monkeypatch, min_c):
    """Every unit at or above the channel threshold (SGCN_TSHIFT_FUSION_MIN_C; 0 = all)
    runs shift_in inside its contraction; units below it keep the two-launch form."""
    import formula
    import shiftgcn
    from shiftgcn import fused, ops
    if min_c is not None:
        monkeypatch.setattr(fused, "TSHIFT_FUSION_MIN_C", min_c)
    calls = {"affine": 0, "plain": 0}
    real = ops.tshift_fwd

    def spy(inp, xpos, ypos, stride, scale=None, **kw):
        # the affine comes as scale/shift, or as a BnStats (possibly a folded finalize)
        aff = scale is not None or kw.get("affine") is not None
        calls["affine" if aff else "plain"] += 1
        return real(inp, xpos, ypos, stride, scale=scale, **kw)

    monkeypatch.setattr(ops, "tshift_fwd", spy)
    m = shiftgcn.Model(num_class=60, num_point=25, num_person=2,
                       graph="graph.ntu_rgb_d.Graph").to(DEV).train()
    x = formula.tensor((2, 3, 16, 25, 2), 5, 1.0).to(DEV)
    m(x).sum().backward()
    torch.cuda.synchronize()
    unfused = sum(getattr(m, f"l{k}").tcn1.in_channels < fused.TSHIFT_FUSION_MIN_C
                  for k in range(1, 11))
    assert calls == {"affine": unfused, "plain": 10}, calls


def _tiny_x_inputs(B, K, M, T, V, seed, sign):
    """xpos all within 2^-25 of 0 (the two-row operand's channels): ``sign`` -1 = all in
    (-2^-25, 0] (exact), 0 = both signs, as shift.py:39's U(-1e-8, 1e-8) init gives."""
    h, w, bias, _, ypos, scale, shift = _inputs(B, K, M, T, V, seed)
    g = torch.Generator().manual_seed(seed + 1)
    xpos = (torch.rand(K, generator=g) - 0.5) * 2e-8
    if sign < 0:
        xpos = -xpos.abs()
    edge = [-2.0 ** -25, -0.0, 0.0, -1e-30]
    if sign >= 0:
        edge += [2.0 ** -26, 1e-30]
    xpos[3:3 + len(edge)] = torch.tensor(edge)
    ypos[10], ypos[11] = 2.0, -1.0                            # integer shifts (dy = 0)
    return h, w, bias, xpos.to(DEV), ypos, scale, shift


TWO_ROW_CASES = [(3, 64, 64, 20, 25), (2, 128, 128, 17, 25), (2, 256, 256, 9, 25),
                 (3, 64, 64, 11, 33)]


@pytest.mark.parametrize("case", TWO_ROW_CASES, ids=["x".join(map(str, c)) for c in TWO_ROW_CASES])
def test_two_row_operand(case):
    """channels with |xpos| < 2^-25 take the two-tap operand
    (rows floor(y), floor(y)+1 of the element's own column). two_row = 1 on xpos <= 0:
    bit-identical to sgcn_tshift_fwd + sgcn_pw_fwd and to the oracle (.cu:49-73 with
    1 - dx == 0); two_row = 2 with both signs: the xpos <= 0 channels still bit-exact vs the
    oracle, the others within 2e-7 x max|tap| (the dropped dx terms weigh < 2^-25 each, plus
    one rounding of the sum; north_star's bar is 1e-5); two_row 0: four taps."""
    from oracle import shift_oracle as so
    from shiftgcn import ops
    from shiftgcn.ops import PlaneView as PV
    B, K, M, T, V = case
    for sign, mode in ((-1, 1), (0, 2), (0, 1), (0, 0)):
        h, w, bias, xpos, ypos, scale, shift = _tiny_x_inputs(*case, seed=sum(case), sign=sign)
        As = ops.tshift_fwd(h, xpos, ypos, 1, scale=scale, shift=shift)
        r1 = torch.empty(B, M, T, V, device=DEV)
        ops.pw_fwd(w, False, bias, PV(As), PV(r1), M, K, T, V, relu=True)
        r2 = torch.empty(B, M, T, V, device=DEV)
        xs = torch.full_like(h, float("nan"))
        ops.pw_fwd_tshift(w, bias, PV(h), xpos, ypos, _St(scale, shift), PV(r2), M, K, T, V,
                          relu=True, x_shifted=xs, two_row=mode)
        r3 = torch.empty(B, M, T, V, device=DEV)   # the contraction of its own operand
        ops.pw_fwd(w, False, bias, PV(xs), PV(r3), M, K, T, V, relu=True)
        torch.cuda.synchronize()
        assert torch.equal(r2, r3), (sign, mode)
        # the oracle: bn affine per element (float32 multiply, then add), then the shift
        hn, sc, sh = h.cpu().numpy(), scale.cpu().numpy(), shift.cpu().numpy()
        aff = (hn * sc[None, :, None, None]).astype(np.float32) + sh[None, :, None, None]
        want = so.shift_forward(aff.astype(np.float32), xpos.cpu().numpy(), ypos.cpu().numpy(), 1)
        got = xs.cpu().numpy()
        xn = xpos.cpu().numpy()
        le0 = xn <= 0
        assert np.array_equal(got[:, le0], want[:, le0]), (sign, mode)
        if mode == 2:
            assert not le0.all()
            err = np.abs(got - want).max() / np.abs(aff).max()
            assert err <= 2e-7, err
            assert ((r2 - r1).abs().max() / r1.abs().max()).item() <= 1e-5
        else:   # exact: every channel, and the contraction too
            assert np.array_equal(got, want), (sign, mode)
            assert torch.equal(r1, r2), (sign, mode)
