"""On-disk feeder (reference feeders/feeder.py:11-95, main.py:235-251):
the .npy clip array + (sample_name, label) pickle, read like the reference, the label file
read without resolving any global, and the device loader's batch order identical to
torch's DataLoader under the same seed."""
import pickle

import numpy as np
import pytest
import torch

from shiftgcn.feeder import DeviceBatchLoader, Feeder, load_labels, loader_order


def _write(tmp_path, n=11, T=6, V=25, M=2, seed=0):
    rng = np.random.default_rng(seed)
    data = rng.standard_normal((n, 3, T, V, M)).astype(np.float32)
    names = [f"S001C001P001R001A{i:03d}.skeleton" for i in range(n)]
    labels = [int(v) for v in rng.integers(0, 60, n)]
    dp, lp = tmp_path / "data.npy", tmp_path / "label.pkl"
    np.save(dp, data)
    with open(lp, "wb") as f:
        pickle.dump((names, labels), f)
    return str(dp), str(lp), data, names, labels


def test_feeder_items_and_len(tmp_path):
    dp, lp, data, names, labels = _write(tmp_path)
    for use_mmap in (True, False):
        f = Feeder(dp, lp, use_mmap=use_mmap)
        assert len(f) == len(labels)
        assert f.sample_name == names
        for i in (0, 5, len(f) - 1):
            x, y, idx = f[i]
            assert isinstance(x, np.ndarray) and x.dtype == np.float32
            assert np.array_equal(x, data[i]) and y == labels[i] and idx == i


def test_feeder_debug_truncates_to_100(tmp_path):
    dp, lp, data, names, labels = _write(tmp_path, n=130, T=2, V=3, M=1)
    f = Feeder(dp, lp, debug=True)
    assert len(f) == 100 and f.data.shape[0] == 100 and f.sample_name == names[:100]


def test_feeder_top_k(tmp_path):
    dp, lp, data, names, labels = _write(tmp_path)
    f = Feeder(dp, lp)
    rng = np.random.default_rng(3)
    score = rng.standard_normal((len(f), 60))
    for k in (1, 5):
        rank = score.argsort()
        want = np.mean([labels[i] in rank[i, -k:] for i in range(len(f))])
        assert f.top_k(score, k) == pytest.approx(want)
    score[np.arange(len(f)), labels] = 100.0
    assert f.top_k(score, 1) == 1.0


def test_labels_python2_pickle_latin1(tmp_path):
    # protocol-2 pickle with a Python 2 byte string holding a non-ASCII byte (0xe9)
    raw = b"\x80\x02(]U\x05S001\xe9a]K\x03at."
    p = tmp_path / "py2.pkl"
    p.write_bytes(raw)
    assert load_labels(str(p)) == (["S001é"], [3])


def test_labels_refuse_globals(tmp_path):
    p = tmp_path / "evil.pkl"
    with open(p, "wb") as f:
        pickle.dump(([print], [1]), f)
    with pytest.raises(pickle.UnpicklingError, match="builtins.print"):
        load_labels(str(p))


def test_feeder_rejects_augmentations(tmp_path):
    dp, lp, *_ = _write(tmp_path)
    with pytest.raises(NotImplementedError):
        Feeder(dp, lp, random_move=True)


@pytest.mark.parametrize("shuffle,drop_last,bs", [(True, True, 3), (False, False, 4),
                                                  (True, False, 5), (False, True, 11)])
def test_loader_order_matches_torch_dataloader(tmp_path, shuffle, drop_last, bs):
    dp, lp, *_ = _write(tmp_path)
    f = Feeder(dp, lp)
    torch.manual_seed(1234)
    want = []
    for _epoch in range(2):
        dl = torch.utils.data.DataLoader(f, batch_size=bs, shuffle=shuffle, drop_last=drop_last)
        want.append([b[2].tolist() for b in dl])
    torch.manual_seed(1234)
    got = [loader_order(len(f), bs, shuffle, drop_last) for _epoch in range(2)]
    assert got == want


def test_device_loader_cpu_batches(tmp_path):
    dp, lp, data, names, labels = _write(tmp_path)
    f = Feeder(dp, lp)
    torch.manual_seed(7)
    dl = torch.utils.data.DataLoader(f, batch_size=4, shuffle=True, drop_last=True)
    want = [(b[0], b[1], b[2]) for b in dl]
    torch.manual_seed(7)
    loader = DeviceBatchLoader(f, 4, shuffle=True, drop_last=True, device="cpu")
    got = list(loader)
    assert len(loader) == len(got) == len(want) == 2
    for (x, y, i), (wx, wy, wi) in zip(got, want):
        assert torch.equal(i, wi) and torch.equal(x, wx) and torch.equal(y, wy)
    # early exit leaves no worker behind
    it = iter(DeviceBatchLoader(f, 2, device="cpu"))
    next(it)
    it.close()


def test_device_loader_shards_global_batches(tmp_path):
    """world_size 2: each global batch of 2*bs (DataLoader order) split between the ranks."""
    dp, lp, *_ = _write(tmp_path, n=17)
    f = Feeder(dp, lp)
    torch.manual_seed(11)
    glob = loader_order(len(f), 6, True, True)
    per_rank = []
    for r in range(2):
        torch.manual_seed(11)
        per_rank.append([i.tolist() for _, _, i in
                         DeviceBatchLoader(f, 3, shuffle=True, drop_last=True, device="cpu",
                                           rank=r, world_size=2)])
    assert len(DeviceBatchLoader(f, 3, drop_last=True, device="cpu", world_size=2)) == 2
    assert [a + b for a, b in zip(*per_rank)] == glob


def test_device_loader_refuses_uneven_shards(tmp_path):
    """world_size > 1 without drop_last would hand the ranks unequal shards of the last
    global batch (a rank with an extra step hangs in the all-reduce): refused up front."""
    dp, lp, *_ = _write(tmp_path, n=17)
    f = Feeder(dp, lp)
    with pytest.raises(ValueError, match="drop_last"):
        DeviceBatchLoader(f, 3, drop_last=False, device="cpu", rank=0, world_size=2)
    assert len(DeviceBatchLoader(f, 3, drop_last=False, device="cpu")) == 6   # 1 rank: fine
