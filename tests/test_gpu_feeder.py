"""DeviceBatchLoader on the GPU: batches land on the device in torch
DataLoader order, bit-identical to the mmap rows, with the copies on a side stream
ordered before the consumer's kernels; a training step consumes them."""
import pickle

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _write(tmp_path, n, T=40, V=25, M=2):
    rng = np.random.default_rng(n)
    data = rng.standard_normal((n, 3, T, V, M)).astype(np.float32)
    labels = [int(v) for v in rng.integers(0, 60, n)]
    np.save(tmp_path / "d.npy", data)
    with open(tmp_path / "l.pkl", "wb") as f:
        pickle.dump(([f"s{i}" for i in range(n)], labels), f)
    return str(tmp_path / "d.npy"), str(tmp_path / "l.pkl"), data, labels


@pytest.mark.parametrize("depth", [1, 3])
def test_device_loader_matches_dataloader(tmp_path, depth):
    from shiftgcn.feeder import DeviceBatchLoader, Feeder
    dp, lp, data, labels = _write(tmp_path, 23)
    f = Feeder(dp, lp)
    torch.manual_seed(3)
    want = [b[2].tolist() for b in torch.utils.data.DataLoader(f, batch_size=4, shuffle=True,
                                                                drop_last=True)]
    torch.manual_seed(3)
    got = []
    for x, y, idx in DeviceBatchLoader(f, 4, shuffle=True, drop_last=True, device="cuda",
                                       depth=depth):
        assert x.is_cuda and y.is_cuda and x.dtype == torch.float32 and y.dtype == torch.int64
        x2 = x * 2.0                      # a consumer kernel on the current stream
        torch.cuda.synchronize()
        i = idx.tolist()
        assert np.array_equal(x.cpu().numpy(), data[i])
        assert np.array_equal(x2.cpu().numpy(), data[i] * 2.0)
        assert y.cpu().tolist() == [labels[k] for k in i]
        got.append(i)
    assert got == want


def test_device_loader_feeds_training_step(tmp_path):
    import shiftgcn
    from shiftgcn import train
    from shiftgcn.feeder import DeviceBatchLoader, Feeder
    dp, lp, data, labels = _write(tmp_path, 6, T=16)
    f = Feeder(dp, lp)
    torch.manual_seed(1)
    model = shiftgcn.Model(num_class=60, num_point=25, num_person=2,
                           graph="graph.ntu_rgb_d.Graph").cuda().train()
    opt = train.build_optimizer(model, base_lr=0.1)
    losses = []
    for x, y, _ in DeviceBatchLoader(f, 2, shuffle=True, drop_last=True):
        losses.append(float(train.train_step(model, opt, x, y)))
    torch.cuda.synchronize()
    assert len(losses) == 3 and all(np.isfinite(losses))
