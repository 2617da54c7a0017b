"""Dispatcher ops (``torch.ops.shiftgcn.tshift_fwd`` / ``tshift_bwd``) and the float64
path (the reference's AT_DISPATCH_FLOATING_TYPES double instantiation, .cu:413).

CPU: the ops are registered, their fake kernels infer shapes on meta tensors, and CPU
tensors raise like the reference's CHECK_INPUT.
GPU: float64 forward / input gradient bit-exact vs the float64 oracle restatement;
``torch.autograd.gradcheck`` of the input gradient (the exact adjoint; the position
gradient is sign-normalised by design, .cu:370-395, so it is not a derivative);
``torch.compile`` (aot_eager: graph capture through the fake kernels + registered autograd,
no code generation) agrees with eager.
"""
import numpy as np
import pytest
import torch

from oracle import shift_oracle as so


def test_ops_registered_and_fake_shapes():
    import shiftgcn  # noqa: F401  (registers the ops)
    x = torch.empty(2, 8, 20, 25, device="meta")
    p = torch.empty(8, device="meta")
    y = torch.ops.shiftgcn.tshift_fwd(x, p, p, 2, True)
    assert y.shape == (2, 8, 10, 25) and y.device.type == "meta"
    gin, gx, gy = torch.ops.shiftgcn.tshift_bwd(y, x, p, p, 2, True)
    assert gin.shape == x.shape and gx.shape == (8,) and gy.shape == (8,)


def test_ops_reject_cpu_tensors():
    import shiftgcn  # noqa: F401
    x = torch.zeros(1, 2, 4, 3)
    p = torch.zeros(2)
    with pytest.raises(RuntimeError, match="must be a CUDA tensor"):
        torch.ops.shiftgcn.tshift_fwd(x, p, p, 1)


def _case(dtype, stride, seed=0, shape=(2, 6, 21, 25)):
    rng = np.random.default_rng(seed + stride)
    B, C, H, W = shape
    x = rng.standard_normal(shape)
    xpos = rng.uniform(-1e-8, 1e-8, C)
    ypos = rng.uniform(-3, 3, C)
    xpos[1], ypos[2] = 1.5, float(H + 1)
    g = rng.standard_normal((B, C, H // stride, W))
    return [a.astype(dtype) for a in (x, xpos, ypos, g)]


@pytest.mark.gpu
@pytest.mark.parametrize("stride", [1, 2])
def test_float64_matches_float64_oracle(stride):
    from shiftgcn import ShiftFunction
    x, xpos, ypos, g = _case(np.float64, stride)
    dev = "cuda"
    xd = torch.from_numpy(x).to(dev).requires_grad_(True)
    xp = torch.from_numpy(xpos).to(dev).requires_grad_(True)
    yp = torch.from_numpy(ypos).to(dev).requires_grad_(True)
    y = ShiftFunction.apply(xd, xp, yp, stride)
    y.backward(torch.from_numpy(g).to(dev))
    assert y.dtype == torch.float64
    ye = ypos if stride == 1 else ypos + 0.5
    assert np.array_equal(y.detach().cpu().numpy(), so.shift_forward(x, xpos, ye, stride))
    rgin, rgx, rgy = so.shift_backward(g, x, xpos, ye, stride)
    assert np.array_equal(xd.grad.cpu().numpy(), rgin)
    assert (yp.grad.cpu().numpy() != rgy).sum() <= 1
    assert (xp.grad.cpu().numpy() != rgx).sum() <= 1


@pytest.mark.gpu
@pytest.mark.parametrize("stride", [1, 2])
def test_gradcheck_input_gradient_float64(stride):
    from shiftgcn import ShiftFunction
    x, xpos, ypos, _ = _case(np.float64, stride, shape=(1, 3, 9, 5))
    dev = "cuda"
    xd = torch.from_numpy(x).to(dev).requires_grad_(True)
    xp = torch.from_numpy(xpos).to(dev)
    yp = torch.from_numpy(ypos).to(dev)
    assert torch.autograd.gradcheck(lambda t: ShiftFunction.apply(t, xp, yp, stride), (xd,),
                                    eps=1e-6, atol=1e-7)


@pytest.mark.gpu
def test_torch_compile_through_dispatcher_ops():
    import shiftgcn
    torch.manual_seed(0)
    m = shiftgcn.Shift(16, stride=2, init_scale=2).to("cuda")
    x = torch.randn(2, 16, 30, 25, device="cuda", requires_grad=True)
    y_e = m(x)
    y_e.sum().backward()
    ge = (x.grad.clone(), m.ypos.grad.clone())
    x.grad = None
    m.ypos.grad = None
    mc = torch.compile(m, backend="aot_eager", fullgraph=True)
    y_c = mc(x)
    y_c.sum().backward()
    assert torch.equal(y_c, y_e)
    assert torch.equal(x.grad, ge[0]) and torch.equal(m.ypos.grad, ge[1])
