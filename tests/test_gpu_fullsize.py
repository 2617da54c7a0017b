"""Full-size parity on the GPU (the BASELINE configs at their real sizes).

The oracle (``oracle/model_oracle.py``, pinned to the reference's own modules by the golden
fixtures) is run on the GPU with the torch-gather temporal shift of ``oracle/torch_shift.py``
in place of ``shift_cuda`` (BASELINE config 1's "naive torch.gather fallback"), in fp32
and in fp64, beside the HIP path:

* config 2 (NTU, x = (64, 3, 300, 25, 2)) and config 3 (MediaPipe, x = (64, 3, 300, 33, 1)):
  one training step at bs=64 each. Every quantity is held to the same relative bar: no
  further from the fp64 eager result than 2x the fp32 eager result is — logits (max abs
  error over max |logit|) and loss with a 1e-5 floor, gradients in norm per parameter
  (median and max over parameters; model-level fp32 gradients through 10 train-mode
  BatchNorm units are ill-conditioned), ypos sign flips vs fp64 2x the fp32 eager's + 2;
  BN running statistics within 1e-4. The achieved errors are printed. At these sizes the
  split-K weight gradients, the 32-bit buffer offsets and the plane-size kernel switches
  (V = 25 and V = 33: 7,500- and 9,900-float planes, 256- vs 512-thread kernels) engage.
* config 4: one 4-stream MediaPipe ensemble batch at bs=256 windows (eval mode): fused
  float64 logits within 1e-4 and fall scores within 1e-5 of the fp64 eager ensemble.
* beyond the 2^29-element operand limit of the contraction kernels (NTU at > ~279 clips
  per GPU): the batch is chunked (ops.pw_fwd / pw_dw) — checked against fp64 torch at the
  op level at NM = 640 (NTU bs=320), and one bs=320 training step runs with finite loss and
  gradients.
"""
import numpy as np
import pytest
import torch

import formula
from oracle import torch_shift as ts
from oracle import model_oracle as mo

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture
def eager_gpu_shift(monkeypatch):
    monkeypatch.setattr(mo.Shift, "function", ts.TorchShiftFunction)


# BASELINE configs 2 and 3: (num_class, V, M, graph)
CONFIGS = {"ntu": (60, 25, 2, "graph.ntu_rgb_d.Graph"),
           "mp": (2, 33, 1, "graph.mediapipe_pose.Graph")}


def _inputs(cfg, bs):
    num_class, V, M, _ = CONFIGS[cfg]
    g = torch.Generator().manual_seed(1000)
    x = torch.randn(bs, 3, 300, V, M, generator=g)
    labels = torch.randint(0, num_class, (bs,), generator=g)
    return x, labels


def _ntu_inputs(bs):
    return _inputs("ntu", bs)


def _run_train(model, x, labels):
    logits = model(x)
    loss = torch.nn.functional.cross_entropy(logits, labels)
    model.zero_grad(set_to_none=True)
    loss.backward()
    torch.cuda.synchronize()
    grads = {n: p.grad.detach().double().cpu() for n, p in model.named_parameters()
             if p.grad is not None}
    bufs = {n: b.detach().double().cpu() for n, b in model.named_buffers()
            if b.dtype.is_floating_point}
    return logits.detach().double().cpu(), float(loss), grads, bufs


@pytest.mark.parametrize("cfg", ["ntu", "mp"])
def test_config2_3_bs64_train_step_matches_eager_reference(eager_gpu_shift, cfg):
    import shiftgcn
    num_class, V, M, graph = CONFIGS[cfg]
    x, labels = _inputs(cfg, 64)
    torch.manual_seed(1)
    ours = shiftgcn.Model(num_class=num_class, num_point=V, num_person=M,
                          graph=graph).to(DEV).train()
    state = {k: v.detach().cpu().clone() for k, v in ours.state_dict().items()}
    lo, losso, go, bo = _run_train(ours, x.to(DEV), labels.to(DEV))
    del ours
    torch.cuda.empty_cache()
    res = {}
    for dt in (torch.float32, torch.float64):
        ref = mo.Model(num_class=num_class, num_point=V, num_person=M)
        ref.load_state_dict(state)
        ref = ref.to(DEV, dt).train()
        res[dt] = _run_train(ref, x.to(DEV, dt), labels.to(DEV))
        del ref
        torch.cuda.empty_cache()
    l32, loss32, g32, b32 = res[torch.float32]
    l64, loss64, g64, b64 = res[torch.float64]

    scale = float(l64.abs().max())
    el_o, el_r = float((lo - l64).abs().max()) / scale, float((l32 - l64).abs().max()) / scale
    ls_o = abs(losso - loss64) / max(1.0, abs(loss64))
    ls_r = abs(loss32 - loss64) / max(1.0, abs(loss64))
    print(f"\n[{cfg}] logits rel err vs fp64: HIP {el_o:.2e}, fp32 eager {el_r:.2e}; "
          f"loss: HIP {ls_o:.2e}, fp32 eager {ls_r:.2e}")
    assert el_o <= max(2 * el_r, 1e-5), (el_o, el_r)
    assert ls_o <= max(2 * ls_r, 1e-5), (ls_o, ls_r)
    for k, b in b64.items():
        err = float((bo[k] - b).abs().max())
        assert err <= 1e-4 * float(b.abs().max()) + 1e-6, (k, err)

    err_o, err_r, flips_o, flips_r = [], [], 0, 0
    for k in sorted(g64):
        if k.endswith("ypos"):
            s64 = torch.sign(g64[k])
            flips_o += int((torch.sign(go[k]) != s64).sum())
            flips_r += int((torch.sign(g32[k]) != s64).sum())
            continue
        n64 = float(g64[k].norm())
        if k.endswith(("Linear_bias", "down.0.bias", "residual.conv.bias")):
            assert float(go[k].abs().max()) < 1e-3, k        # zero by construction (pre-BN)
            continue
        if n64 == 0.0:
            assert float(go[k].abs().max()) == 0.0, k         # xpos
            continue
        err_o.append(float((go[k] - g64[k]).norm()) / n64)
        err_r.append(float((g32[k] - g64[k]).norm()) / n64)
    err_o, err_r = np.array(err_o), np.array(err_r)
    print(f"[{cfg}] grad rel err vs fp64 (median / max over params): HIP "
          f"{np.median(err_o):.2e} / {err_o.max():.2e}, fp32 eager {np.median(err_r):.2e} / "
          f"{err_r.max():.2e}; ypos sign flips {flips_o} vs {flips_r}")
    assert np.median(err_o) <= 2 * np.median(err_r) + 1e-5, (np.median(err_o), np.median(err_r))
    assert err_o.max() <= 2 * err_r.max() + 1e-5, (err_o.max(), err_r.max())
    assert flips_o <= 2 * flips_r + 2, (flips_o, flips_r)


def _eager_streams(joint, parent):
    """derive_modalities (inference_pipeline.py:284-309) on the device, batched."""
    bone = joint - joint[:, :, :, parent.long(), :]
    T = joint.shape[2]

    def motion(a):
        out = torch.zeros_like(a)
        out[:, :, :T - 1] = a[:, :, 1:] - a[:, :, :T - 1]
        return out

    return [joint, bone, motion(joint), motion(bone)]


def test_config4_ensemble_bs256_matches_eager_reference(eager_gpu_shift):
    import shiftgcn
    from shiftgcn.ensemble import Ensemble
    models = []
    for k in range(4):
        m = shiftgcn.Model(num_class=2, num_point=33, num_person=1,
                           graph="graph.mediapipe_pose.Graph")
        formula.fill_state(m, seed=500 + k)
        models.append(m.to(DEV).eval())
    ens = Ensemble(models).to(DEV)
    g = torch.Generator().manual_seed(2000)
    x = torch.randn(256, 3, 300, 33, 1, generator=g).to(DEV)
    scores, fused = ens(x)
    torch.cuda.synchronize()
    scores, fused = scores.cpu(), fused.cpu()
    with torch.no_grad():
        acc = torch.zeros(256, 2, dtype=torch.float64, device=DEV)
        streams = _eager_streams(x.double(), ens.parent)
        for k, (m, s) in enumerate(zip(models, streams)):
            ref = mo.Model(num_class=2, num_point=33, num_person=1)
            ref.load_state_dict(m.state_dict())
            ref = ref.to(DEV, torch.float64).eval()
            acc += float(np.float32(ens.weights[k])) * ref(s)
            del ref
        e = torch.exp(acc - acc.max(dim=1, keepdim=True).values)
        sref = (e[:, 1] / e.sum(dim=1)).cpu()
    acc = acc.cpu()
    assert float((fused - acc).abs().max()) <= 1e-4 * float(acc.abs().max())
    assert float((scores - sref).abs().max()) <= 1e-5


def test_pointwise_batch_chunking_beyond_32bit_offsets():
    """NM = 640 (NTU bs=320) at l5's tcn contraction: 640*128*300*25 = 614 M elements per
    operand > 2^29, so ops.pw_fwd / pw_dw split the batch; checked against fp64 torch."""
    from shiftgcn import ops
    from shiftgcn.ops import PlaneView as PV
    B, K, M, T, V = 640, 128, 128, 300, 25
    assert B * K * T * V >= ops.PW_MAX_ELEMS
    torch.manual_seed(0)
    x = torch.randn(B, K, T, V, device=DEV)
    w = torch.randn(M, K, device=DEV) / K ** 0.5
    bias = torch.randn(M, device=DEV)
    y = torch.empty(B, M, T, V, device=DEV)
    ops.pw_fwd(w, False, bias, PV(x), PV(y), M, K, T, V)
    # fp64 reference on sampled samples (first, last, and both sides of a chunk seam)
    bc = ops._batch_chunk([(PV(x), K), (PV(y), M)], B, T, V)
    assert bc < B
    for b in sorted({0, bc - 1, bc, B - 1}):
        ref = torch.einsum("mk,ktv->mtv", w.double(), x[b].double()) + bias.double()[:, None, None]
        err = float((y[b].double() - ref).abs().max())
        assert err <= 1e-5 * float(ref.abs().max()), (b, err)
    del y
    g = torch.randn(B, M, T, V, device=DEV) * 1e-2
    dw = torch.empty(M, K, device=DEV)
    db = torch.empty(M, device=DEV)
    ops.pw_dw(PV(g), PV(x), dw, M, K, T, V, dbias=db)
    ref_dw = torch.zeros(M, K, dtype=torch.float64, device=DEV)
    for b0 in range(0, B, 64):
        ref_dw += torch.einsum("bmn,bkn->mk", g[b0:b0 + 64].double().flatten(2),
                               x[b0:b0 + 64].double().flatten(2))
    ref_db = g.double().sum(dim=(0, 2, 3))
    assert float((dw.double() - ref_dw).abs().max()) <= 1e-5 * float(ref_dw.abs().max())
    assert float((db.double() - ref_db).abs().max()) <= 1e-5 * float(ref_db.abs().max())


def test_ntu_bs320_train_step_runs_chunked():
    import shiftgcn
    from shiftgcn import ops, train
    calls = {"chunked": 0}
    real = ops._batch_chunk

    def spy(views, B, T, V):
        bc = real(views, B, T, V)
        calls["chunked"] += int(bc < B)
        return bc

    ops._batch_chunk = spy
    try:
        torch.manual_seed(1)
        m = shiftgcn.Model(num_class=60, num_point=25, num_person=2,
                           graph="graph.ntu_rgb_d.Graph").to(DEV).train()
        opt = train.build_optimizer(m, base_lr=0.1)
        x, labels = _ntu_inputs(320)
        loss = train.train_step(m, opt, x.to(DEV), labels.to(DEV))
        torch.cuda.synchronize()
    finally:
        ops._batch_chunk = real
    assert calls["chunked"] > 0
    assert np.isfinite(float(loss))
    for n, p in m.named_parameters():
        if p.grad is not None:
            assert bool(torch.isfinite(p.grad).all()), n
