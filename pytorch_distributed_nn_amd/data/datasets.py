"""Datasets, readers and the prefetching loader (see package docstring)."""
from __future__ import annotations

import os
import queue
import threading
from pathlib import Path

import numpy as np
import torch

MNIST_SEED = 66478      # pytorch_code/mnist/mnist.py:35


class DataSet:
    """Arrays + epoch-wrapping ``next_batch`` with a reshuffle at every epoch boundary."""

    def __init__(self, images: np.ndarray, labels: np.ndarray, seed: int = MNIST_SEED, shuffle: bool = True):
        assert len(images) == len(labels)
        self.images, self.labels = images, labels
        self.num_examples = len(images)
        self.epochs_completed = 0
        self._index = 0
        self._rng = np.random.RandomState(seed)
        self._shuffle = shuffle
        if shuffle:
            self._perm()

    def _perm(self):
        p = self._rng.permutation(self.num_examples)
        self.images, self.labels = self.images[p], self.labels[p]

    def next_batch(self, batch_size: int):
        start = self._index
        if start + batch_size > self.num_examples:
            # finish the epoch with the remaining rows, reshuffle, continue (mnist.py:102-131)
            rest = self.num_examples - start
            xi, yi = self.images[start:], self.labels[start:]
            self.epochs_completed += 1
            if self._shuffle:
                self._perm()
            self._index = batch_size - rest
            return (np.concatenate([xi, self.images[: self._index]]),
                    np.concatenate([yi, self.labels[: self._index]]))
        self._index += batch_size
        return self.images[start:self._index], self.labels[start:self._index]

    def skip(self, batch_size: int, n: int = 1):
        """Advance past ``n`` batches exactly as ``n`` calls of :meth:`next_batch` would (same reshuffles at the
        same epoch boundaries, same RNG draws), without gathering any rows."""
        for _ in range(n):
            start = self._index
            if start + batch_size > self.num_examples:
                self.epochs_completed += 1
                if self._shuffle:
                    self._perm()
                self._index = batch_size - (self.num_examples - start)
            else:
                self._index += batch_size

    def __len__(self):
        return self.num_examples


# ------------------------------------------------------------------------------------------------ MNIST
def write_mnist_like(dir_, n_train=256, n_test=64, seed=0):
    """Write synthetic MNIST-format IDX files (same magic numbers/shapes) — used by tests and offline runs."""
    from ..utils.native import idx_write
    d = Path(dir_)
    d.mkdir(parents=True, exist_ok=True)
    rng = np.random.RandomState(seed)
    for split, n in (("train", n_train), ("t10k", n_test)):
        labels = rng.randint(0, 10, n).astype(np.uint8)
        imgs = (rng.rand(n, 28, 28) * 64).astype(np.uint8)
        for i, l in enumerate(labels):     # a learnable pattern: a bright column per class
            imgs[i, 4:24, 2 + 2 * l] = 255
        idx_write(d / f"{split}-images-idx3-ubyte", imgs)
        idx_write(d / f"{split}-labels-idx1-ubyte", labels)
    return d


def read_mnist(dir_, reshape: bool = True, flat: bool = False, one_hot: bool = False, seed: int = MNIST_SEED):
    """-> (train DataSet, test DataSet).  Files: {train,t10k}-{images-idx3,labels-idx1}-ubyte."""
    from ..utils.native import idx_read
    d = Path(dir_)
    out = []
    for split in ("train", "t10k"):
        imgs = idx_read(d / f"{split}-images-idx3-ubyte").astype(np.float32) / 255.0 - 0.5
        labels = idx_read(d / f"{split}-labels-idx1-ubyte").astype(np.int64)
        if flat:
            imgs = imgs.reshape(len(imgs), -1)
        elif reshape:
            imgs = imgs.reshape(len(imgs), 1, 28, 28)
        if one_hot:
            labels = np.eye(10, dtype=np.float32)[labels]
        out.append(DataSet(imgs, labels, seed=seed, shuffle=split == "train"))
    return out[0], out[1]


# ------------------------------------------------------------------------------------------------ CIFAR-10
def read_cifar10(dir_, normalize: bool = True, seed: int = 0):
    """CIFAR-10 binary version: each record = 1 label byte + 3072 pixel bytes (R plane, G plane, B plane).
    Returns (train DataSet, test DataSet) with NCHW float32 images."""
    d = Path(dir_)

    def load(files):
        raw = np.concatenate([np.fromfile(d / f, dtype=np.uint8) for f in files])
        raw = raw.reshape(-1, 3073)
        labels = raw[:, 0].astype(np.int64)
        imgs = raw[:, 1:].reshape(-1, 3, 32, 32).astype(np.float32) / 255.0   # planes are already CHW
        if normalize:
            mean = np.array([0.4914, 0.4822, 0.4465], np.float32)[:, None, None]
            std = np.array([0.2470, 0.2435, 0.2616], np.float32)[:, None, None]
            imgs = (imgs - mean) / std
        return imgs, labels

    tr = load([f"data_batch_{i}.bin" for i in range(1, 6) if (d / f"data_batch_{i}.bin").exists()])
    te = load(["test_batch.bin"]) if (d / "test_batch.bin").exists() else tr
    return DataSet(*tr, seed=seed), DataSet(*te, seed=seed, shuffle=False)


def augment_crop_flip(x: np.ndarray, pad: int = 4, rng=None) -> np.ndarray:
    """Random crop with zero padding + horizontal flip (reference cifar10.py:458-494), NCHW batch."""
    rng = rng or np.random
    n, c, h, w = x.shape
    xp = np.pad(x, ((0, 0), (0, 0), (pad, pad), (pad, pad)))
    out = np.empty_like(x)
    for i in range(n):
        dy, dx = rng.randint(0, 2 * pad + 1, 2)
        img = xp[i, :, dy:dy + h, dx:dx + w]
        out[i] = img[:, :, ::-1] if rng.rand() < 0.5 else img
    return out


# ------------------------------------------------------------------------------------------------ synthetic
class SyntheticDataset:
    """Random inputs/labels of a given shape, generated once on the target device (benchmarks)."""

    def __init__(self, shape, num_classes=1000, n_batches=2, batch_size=256, device="cpu", dtype=torch.float32,
                 seed=0):
        g = torch.Generator(device="cpu").manual_seed(seed)
        self.batches = []
        for _ in range(n_batches):
            x = torch.randn(batch_size, *shape, generator=g).to(device=device, dtype=dtype)
            y = torch.randint(0, num_classes, (batch_size,), generator=g).to(device)
            self.batches.append((x, y))
        self._i = 0

    def next_batch(self, batch_size=None):
        b = self.batches[self._i % len(self.batches)]
        self._i += 1
        return b

    def __iter__(self):
        while True:
            yield self.next_batch()


class SyntheticTokens:
    """Random token sequences for language models: (input ids, next-token targets)."""

    def __init__(self, vocab, seq_len, batch_size, device="cpu", n_batches=2, seed=0):
        g = torch.Generator(device="cpu").manual_seed(seed)
        self.batches = []
        for _ in range(n_batches):
            t = torch.randint(0, vocab, (batch_size, seq_len + 1), generator=g).to(device)
            self.batches.append((t[:, :-1].contiguous(), t[:, 1:].contiguous()))
        self._i = 0

    def next_batch(self, batch_size=None):
        b = self.batches[self._i % len(self.batches)]
        self._i += 1
        return b

    def __iter__(self):
        while True:
            yield self.next_batch()


# ------------------------------------------------------------------------------------------------ loader
def _loader_worker(images, labels, transform, index_q, data_q, wid, seed, rank=0):
    """Worker process (PT-11 my_data_loader.py:37-53): (seq, indices) -> (seq, x, y), gathered and
    transformed in this process; None ends it.  ``images``/``labels`` arrive as shared-memory tensors (one
    copy per node, not one pickled copy per worker per rank); the augmentation stream is seeded per rank
    AND worker, so ranks do not draw identical random crops/flips."""
    if isinstance(images, torch.Tensor):
        images, labels = images.numpy(), labels.numpy()
    np.random.seed((seed + 1000 * rank + wid) % (2 ** 32))
    while True:
        job = index_q.get()
        if job is None:
            break
        seq, idx = job
        x, y = images[idx], labels[idx]
        if transform is not None:
            x = transform(x)
        data_q.put((seq, np.ascontiguousarray(x), np.ascontiguousarray(y)))


class DataLoader:
    """Batches from a :class:`DataSet`, sharded by rank, prefetched into pinned memory and copied to the
    device asynchronously on a side stream.

    ``rank``/``world`` shard the sample stream (each rank draws every world-th batch), so DDP ranks see
    disjoint data like torch's DistributedSampler.

    ``num_workers = 0``: one background thread draws batches (epoch-wrapping ``next_batch``).
    ``num_workers > 0`` (PT-11, pytorch_code/data_loader_ops/my_data_loader.py:37-53, 137-251): the main
    process keeps the sampler (a per-epoch permutation, seeded, sharded by rank) and feeds ``(seq, indices)``
    jobs round-robin to worker PROCESSES through per-worker index queues; the workers gather and transform
    the samples (the CPU-heavy part: augmentation) and return ``(seq, x, y)`` on one data queue; batches are
    reassembled in sequence order (out-of-order arrivals wait in a reorder buffer, :185-211) before
    pinning."""

    def __init__(self, dataset: DataSet, batch_size: int, device="cpu", prefetch: int = 4, rank: int = 0,
                 world: int = 1, transform=None, drop_last: bool = True, num_workers: int = 0, seed: int = 0):
        self.ds, self.bs = dataset, batch_size
        self.device = torch.device(device)
        self.rank, self.world = rank, world
        self.transform = transform
        self.q: queue.Queue = queue.Queue(maxsize=prefetch)
        self._stop = False
        self._pin = self.device.type == "cuda"
        self.num_workers = num_workers
        self._procs = []
        self._skip_pending = self._produced = self._consumed = 0
        if num_workers > 0:
            import torch.multiprocessing as mp
            ctx = mp.get_context("spawn")          # workers never touch the GPU; spawn is fork-safe with HIP
            self._index_qs = [ctx.Queue() for _ in range(num_workers)]
            self._data_q = ctx.Queue(maxsize=max(2, prefetch) * num_workers)
            # shared-memory tensors pickle as handles: every worker maps the same pages
            shm_x = torch.from_numpy(np.ascontiguousarray(dataset.images)).share_memory_()
            shm_y = torch.from_numpy(np.ascontiguousarray(dataset.labels)).share_memory_()
            for w in range(num_workers):
                p = ctx.Process(target=_loader_worker, args=(shm_x, shm_y, transform, self._index_qs[w],
                                                             self._data_q, w, seed, rank), daemon=True)
                p.start()
                self._procs.append(p)
            self._sampler_rng = np.random.RandomState(seed)
            self._perm, self._pos = self._sampler_rng.permutation(len(dataset)), 0
            self._send_seq, self._recv_seq, self._reorder = 0, 0, {}
            self._lock = threading.Lock()
            for _ in range(max(2, prefetch) * num_workers):      # keep every worker busy
                self._dispatch()
        if not hasattr(self, "_lock"):
            self._lock = threading.Lock()     # held while a batch is drawn: skip() moves the sampler in between
        self._thread = threading.Thread(target=self._worker if num_workers == 0 else self._collector, daemon=True)
        self._thread.start()
        self._stream = torch.cuda.Stream(self.device) if self._pin else None

    # -------------------------------------------------------------- multiprocess path
    def _next_indices(self):
        """The next batch of this rank: batches are dealt round-robin over ranks from one permutation per
        epoch (a partial batch at the epoch end wraps into the next permutation)."""
        out = []
        need = self.bs * self.world
        while len(out) < need:
            take = min(need - len(out), len(self._perm) - self._pos)
            out.extend(self._perm[self._pos:self._pos + take].tolist())
            self._pos += take
            if self._pos == len(self._perm):
                self._perm, self._pos = self._sampler_rng.permutation(len(self.ds)), 0
        return np.asarray(out[self.rank * self.bs:(self.rank + 1) * self.bs])

    def _dispatch(self):
        with self._lock:
            while self._skip_pending:         # batches a resume fast-forwards over: drawn, never built
                self._skip_pending -= 1
                self._next_indices()
            self._index_qs[self._send_seq % self.num_workers].put((self._send_seq, self._next_indices()))
            self._send_seq += 1
            self._produced += 1

    def _collector(self):
        while not self._stop:
            while self._recv_seq not in self._reorder:
                try:
                    seq, x, y = self._data_q.get(timeout=1.0)
                except queue.Empty:
                    if self._stop:
                        return
                    continue
                self._reorder[seq] = (x, y)
            x, y = self._reorder.pop(self._recv_seq)
            self._recv_seq += 1
            xt, yt = torch.from_numpy(x), torch.from_numpy(y)
            if self._pin:
                xt, yt = xt.pin_memory(), yt.pin_memory()
            self.q.put((xt, yt))
            self._dispatch()                  # after the put: a skip() holding the lock can always drain the queue

    # -------------------------------------------------------------- thread path
    def _worker(self):
        while not self._stop:
            with self._lock:
                self._produced += 1
                self.ds.skip(self.bs, self.rank)
                x, y = self.ds.next_batch(self.bs)
                self.ds.skip(self.bs, self.world - 1 - self.rank)
                if self.transform is not None:
                    x = self.transform(x)
                xt, yt = torch.from_numpy(np.ascontiguousarray(x)), torch.from_numpy(np.ascontiguousarray(y))
            if self._pin:
                xt, yt = xt.pin_memory(), yt.pin_memory()
            self.q.put((xt, yt))

    def skip(self, n: int):
        """Fast-forward past the next ``n`` batches of this rank (a resumed run re-aligning its data stream)
        without building them: batches already drawn (prefetched, or in a worker) are dropped as they arrive,
        the rest are only drawn from the sampler -- no gather, no augmentation, no pinning, no host-to-device
        copy.  The producers draw under ``_lock``, so the sampler moves past the skipped batches before
        any later batch is drawn."""
        n = int(n)
        if n <= 0:
            return
        with self._lock:
            inflight = self._produced - self._consumed
            direct = min(n, inflight)
            self._consumed += n
            self._produced += n - direct
            if self.num_workers == 0:
                self.ds.skip(self.bs, (n - direct) * self.world)
            else:
                self._skip_pending += n - direct
        for _ in range(direct):               # drawn before the skip, so ahead of it in order: dropped on arrival
            self.q.get()

    def next_batch(self, batch_size=None):
        x, y = self.q.get()
        self._consumed += 1
        if self._pin:
            with torch.cuda.stream(self._stream):
                x = x.to(self.device, non_blocking=True)
                y = y.to(self.device, non_blocking=True)
            torch.cuda.current_stream(self.device).wait_stream(self._stream)
            x.record_stream(torch.cuda.current_stream(self.device))
            y.record_stream(torch.cuda.current_stream(self.device))
        return x, y

    def __iter__(self):
        while True:
            yield self.next_batch()

    def __len__(self):
        return len(self.ds) // (self.bs * self.world)

    def close(self):
        self._stop = True
        for q in getattr(self, "_index_qs", []):
            q.put(None)
        for p in self._procs:
            p.join(timeout=5)
            if p.is_alive():
                p.kill()


class DeviceDataLoader:
    """The whole dataset resident in device memory; batches are gathered on the device (no host staging).

    For synthetic data and datasets that fit with room to spare in one MI355X's 288 GB (MNIST is 47 MB as
    bf16, CIFAR-10 150 MB): a host loader must move every batch over PCIe (ResNet-50 at 11.5k img/s wants
    ~3.5 GB/s of bf16 224x224 images after the host has gathered and pinned them), this one reads HBM.  Same
    sampling contract as :class:`DataLoader`: a seeded permutation per epoch (drawn on the device), batches
    dealt round-robin over ``world`` ranks, epoch-wrapping; :meth:`skip` is O(1) per batch."""

    def __init__(self, dataset: DataSet, batch_size: int, device, rank: int = 0, world: int = 1, seed: int = 0,
                 dtype=None):
        self.device = torch.device(device)
        x = torch.from_numpy(np.ascontiguousarray(dataset.images))
        self.x = x.to(self.device, dtype=dtype or x.dtype)
        self.y = torch.from_numpy(np.ascontiguousarray(dataset.labels)).to(self.device)
        self.n, self.bs, self.rank, self.world = len(dataset), batch_size, rank, world
        self.gen = torch.Generator(device=self.device).manual_seed(seed)
        self.perm, self.pos = self._new_perm(), 0

    def _new_perm(self):
        return torch.randperm(self.n, generator=self.gen, device=self.device)

    def _next_global(self):
        """Indices (device tensor) of the next global batch of bs * world samples."""
        need, parts = self.bs * self.world, []
        while need:
            take = min(need, self.n - self.pos)
            parts.append(self.perm[self.pos:self.pos + take])
            self.pos += take
            need -= take
            if self.pos == self.n:
                self.perm, self.pos = self._new_perm(), 0
        return parts[0] if len(parts) == 1 else torch.cat(parts)

    def next_batch(self, batch_size=None):
        idx = self._next_global()[self.rank * self.bs:(self.rank + 1) * self.bs]
        return self.x.index_select(0, idx), self.y.index_select(0, idx)

    def skip(self, n: int):
        for _ in range(int(n)):
            self._next_global()

    def __iter__(self):
        while True:
            yield self.next_batch()

    def __len__(self):
        return self.n // (self.bs * self.world)

    def close(self):
        pass


class MNISTDataset(torch.utils.data.Dataset):
    """torch Dataset over a MNIST :class:`DataSet` (PT-12 datasets/__init__.py:5-27)."""

    def __init__(self, dataset: DataSet, transform=None, target_transform=None):
        self.ds, self.transform, self.target_transform = dataset, transform, target_transform

    def __getitem__(self, i):
        x, y = torch.from_numpy(np.asarray(self.ds.images[i])), int(self.ds.labels[i])
        if self.transform:
            x = self.transform(x)
        if self.target_transform:
            y = self.target_transform(y)
        return x, y

    def __len__(self):
        return len(self.ds)

    def next_batch(self, batch_size):
        x, y = self.ds.next_batch(batch_size)
        return torch.from_numpy(x), torch.from_numpy(np.asarray(y))


class Cifar10Dataset(MNISTDataset):
    """torch Dataset over a CIFAR-10 :class:`DataSet` (PT-12 datasets/__init__.py:29-51)."""


def dataset_from_args(name: str, data_dir: str | None, synthetic: bool, device, batch_size: int, model_name: str):
    """(train, test) sources for the CLI: real files when present, otherwise synthetic of the right shape."""
    name = name.upper()
    if not synthetic and data_dir and os.path.isdir(data_dir):
        if name == "MNIST":
            flat = model_name.lower().startswith("mlp")
            return read_mnist(data_dir, flat=flat)
        if name == "CIFAR10":
            return read_cifar10(data_dir)
    shape = {"MNIST": (1, 28, 28), "CIFAR10": (3, 32, 32), "IMAGENET": (3, 224, 224)}[name]
    if model_name.lower().startswith("mlp"):
        shape = (int(np.prod(shape)),)
    nc = 1000 if name == "IMAGENET" else 10
    n = 4 * batch_size
    rng = np.random.RandomState(0)
    centers = rng.randn(nc, *shape).astype(np.float32)
    y = rng.randint(0, nc, n)
    x = (centers[y] + 0.5 * rng.randn(n, *shape)).astype(np.float32)
    return DataSet(x, y.astype(np.int64)), DataSet(x[: 2 * batch_size], y[: 2 * batch_size].astype(np.int64),
                                                   shuffle=False)
