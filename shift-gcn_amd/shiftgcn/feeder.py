"""On-disk clip feeder: the reference's ``.npy`` + label-pickle format
(``feeders/feeder.py:11-95``, written by ``data_gen/ntu_gendata.py:137-139``), fed to the
device without stalling the compute stream.

* :class:`Feeder` — drop-in for ``feeders.feeder.Feeder``: same constructor, ``len``,
  ``__getitem__ -> (clip, label, index)`` and ``top_k`` (so ``torch.utils.data.DataLoader``
  and ``main.py``'s eval loop work unchanged). The clip array ``(N, C, T, V, M)`` float32
  is memory-mapped (``use_mmap``); the ``(sample_name, label)`` pickle is read with a
  restricted unpickler that resolves NO globals (plain lists/tuples/str/int only), so a
  label file cannot execute code. The augmentations of ``feeders/tools.py`` are off in
  every reference config (``config/*/train_*.yaml``) and are not provided.
* :class:`DeviceBatchLoader` — the training/eval batch stream on the GPU: the next
  batches' rows are gathered from the mmap into pinned host buffers by a worker thread
  (numpy's gather releases the GIL) and copied host->device on a dedicated copy stream,
  ``depth`` batches ahead; the compute stream waits on an event per batch, never on the
  host. Batch order is identical to ``DataLoader(feeder, batch_size, shuffle, drop_last)``
  under the same global torch seed (``main.py:235-251``).
"""
from __future__ import annotations

import collections
import io
import pickle
import queue
import threading

import numpy as np
import torch


class _NoGlobalsUnpickler(pickle.Unpickler):
    """Unpickler for the label file: containers and scalars only (no class lookups)."""

    def find_class(self, module, name):
        raise pickle.UnpicklingError(
            f"label file references {module}.{name}: only plain lists/tuples/str/int are "
            "accepted")


def load_labels(label_path):
    """``(sample_name, label)`` from a reference label pickle (``feeder.py:44-52``: Python 3
    pickles, and Python 2 pickles decoded as latin1)."""
    with open(label_path, "rb") as f:
        raw = f.read()
    try:
        obj = _NoGlobalsUnpickler(io.BytesIO(raw)).load()
    except UnicodeDecodeError:
        obj = _NoGlobalsUnpickler(io.BytesIO(raw), encoding="latin1").load()
    if not (isinstance(obj, (tuple, list)) and len(obj) == 2):
        raise ValueError("label file must hold (sample_name, label)")
    sample_name, label = obj
    return list(sample_name), [int(v) for v in label]


class Feeder(torch.utils.data.Dataset):
    """``feeders/feeder.py:11-95`` (mmap'd clips + label pickle)."""

    def __init__(self, data_path, label_path, random_choose=False, random_shift=False,
                 random_move=False, window_size=-1, normalization=False, debug=False,
                 use_mmap=True):
        if random_choose or random_shift or random_move or window_size > 0 or normalization:
            raise NotImplementedError(
                "feeder augmentations (random_choose/shift/move, window_size, normalization) "
                "are not provided: every reference config runs with them off")
        self.debug = debug
        self.data_path = data_path
        self.label_path = label_path
        self.use_mmap = use_mmap
        self.load_data()

    def load_data(self):
        self.sample_name, self.label = load_labels(self.label_path)
        self.data = np.load(self.data_path, mmap_mode="r" if self.use_mmap else None,
                            allow_pickle=False)
        if self.data.ndim != 5:
            raise ValueError(f"clip array must be (N, C, T, V, M), got {self.data.shape}")
        if self.debug:   # feeder.py:57-60
            self.label = self.label[0:100]
            self.data = self.data[0:100]
            self.sample_name = self.sample_name[0:100]
        if len(self.label) != self.data.shape[0]:
            raise ValueError(f"{len(self.label)} labels for {self.data.shape[0]} clips")

    def __len__(self):
        return len(self.label)

    def __iter__(self):
        return self

    def __getitem__(self, index):
        return np.array(self.data[index]), self.label[index], index

    def top_k(self, score, top_k):
        """Fraction of samples whose label is among the top_k scores (``feeder.py:92-95``)."""
        rank = np.asarray(score).argsort()
        hit = [lab in rank[i, -top_k:] for i, lab in enumerate(self.label)]
        return sum(hit) * 1.0 / len(hit)


def loader_order(n, batch_size, shuffle, drop_last, generator=None):
    """Index batches in the order ``torch.utils.data.DataLoader(dataset, batch_size,
    shuffle, drop_last)`` (num_workers=0) yields them: one draw of the global generator
    for the iterator's base seed, then ``RandomSampler``'s seed draw and ``randperm``."""
    torch.empty((), dtype=torch.int64).random_(generator=generator)   # _BaseDataLoaderIter
    if shuffle:
        if generator is None:
            seed = int(torch.empty((), dtype=torch.int64).random_().item())
            generator = torch.Generator()
            generator.manual_seed(seed)
        order = torch.randperm(n, generator=generator).tolist()
    else:
        order = list(range(n))
    batches = [order[i:i + batch_size] for i in range(0, n, batch_size)]
    if drop_last and batches and len(batches[-1]) < batch_size:
        batches.pop()
    return batches


class DeviceBatchLoader:
    """Iterate ``(clips, labels, indices)`` batches of a :class:`Feeder` on ``device``,
    prefetched ``depth`` batches ahead (pinned staging + a copy stream + events)."""

    def __init__(self, feeder: Feeder, batch_size, shuffle=False, drop_last=False,
                 device="cuda", depth=2, generator=None, rank=0, world_size=1):
        self.feeder = feeder
        self.batch_size = int(batch_size)
        # data-parallel shard: every rank draws the same global order (same seed) of
        # batch_size*world_size batches and takes its slice of each
        self.rank, self.world_size = int(rank), int(world_size)
        if self.world_size > 1 and not drop_last:
            # a short last global batch would give the ranks unequal (or empty) shards: a
            # rank with an extra step then waits forever in the gradient all-reduce, and the
            # 1/world mean of GradAllReduce assumes equal shards
            raise ValueError("DeviceBatchLoader: world_size > 1 needs drop_last=True "
                             "(every rank must run the same number of equal batches)")
        self.shuffle, self.drop_last = shuffle, drop_last
        self.device = torch.device(device)
        self.depth = max(1, int(depth))
        self.generator = generator

    def __len__(self):
        n, gb = len(self.feeder), self.batch_size * self.world_size
        return n // gb if self.drop_last else -(-n // gb)

    def __iter__(self):
        bs, r = self.batch_size, self.rank
        batches = loader_order(len(self.feeder), bs * self.world_size, self.shuffle,
                               self.drop_last, self.generator)
        if self.world_size > 1:
            batches = [b[r * bs:(r + 1) * bs] for b in batches]   # full global batches
        if not batches:
            return
        data = self.feeder.data
        labels = np.asarray(self.feeder.label, dtype=np.int64)
        cuda = self.device.type == "cuda"
        shape = (self.batch_size,) + tuple(data.shape[1:])
        nbuf = self.depth + 2
        hx = [torch.empty(shape, dtype=torch.float32, pin_memory=cuda) for _ in range(nbuf)]
        hy = [torch.empty((self.batch_size,), dtype=torch.int64, pin_memory=cuda)
              for _ in range(nbuf)]
        free, ready, stop = queue.Queue(), queue.Queue(), threading.Event()
        for k in range(nbuf):
            free.put(k)

        def gather():   # worker: mmap rows -> pinned buffer k (np.take releases the GIL)
            try:
                for idx in batches:
                    k = free.get()
                    if k is None or stop.is_set():
                        return
                    ia = np.asarray(idx, dtype=np.int64)
                    np.take(data, ia, axis=0, out=hx[k].numpy()[:len(idx)])
                    hy[k].numpy()[:len(idx)] = labels[ia]
                    ready.put((k, idx))
            except BaseException as e:   # re-raised in the consumer
                ready.put(e)

        th = threading.Thread(target=gather, daemon=True)
        th.start()
        copy_stream = torch.cuda.Stream(self.device) if cuda else None
        pending = collections.deque()    # copies issued, not yet handed out
        inflight = collections.deque()   # (k, event): staging buffer k may still be read

        def recycle(block):
            while inflight and (inflight[0][1].query() or block):
                k, ev = inflight.popleft()
                ev.synchronize()
                free.put(k)
                block = False

        def issue():
            if cuda and len(inflight) >= nbuf - 1:
                recycle(block=True)      # keep a staging buffer for the worker (no deadlock)
            item = ready.get()
            if isinstance(item, BaseException):
                raise item
            k, idx = item
            b = len(idx)
            if cuda:
                with torch.cuda.stream(copy_stream):
                    x = hx[k][:b].to(self.device, non_blocking=True)
                    y = hy[k][:b].to(self.device, non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(copy_stream)
                inflight.append((k, ev))
            else:
                x, y, ev = hx[k][:b].clone(), hy[k][:b].clone(), None
                free.put(k)
            pending.append((x, y, idx, ev))

        try:
            n_issued = 0
            while n_issued < min(self.depth, len(batches)):
                issue()
                n_issued += 1
            for _ in batches:
                x, y, idx, ev = pending.popleft()
                if cuda:
                    cur = torch.cuda.current_stream(self.device)
                    cur.wait_event(ev)
                    x.record_stream(cur)
                    y.record_stream(cur)
                if n_issued < len(batches):   # next copy overlaps this batch's compute
                    issue()
                    n_issued += 1
                if cuda:
                    recycle(block=False)
                yield x, y, torch.tensor(idx, dtype=torch.int64)
        finally:
            stop.set()
            free.put(None)
            for _, ev in inflight:
                ev.synchronize()
            th.join(timeout=30)
