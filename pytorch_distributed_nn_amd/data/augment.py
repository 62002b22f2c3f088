"""Data augmentation helpers of the reference loaders, vectorised with NumPy, for NCHW batches
(``N x C x H x W``; flat MNIST rows ``N x 784`` are reshaped to 1 x 28 x 28 where a spatial op needs it).

Behaviour parity (PT-13 pytorch_code/mnist/mnist.py:216-381, PT-14 pytorch_code/cifar10/cifar10.py:201-264,
458-494):  random crop with zero padding, CIFAR crop + horizontal flip, per-image whitening with the
adjusted standard deviation max(std, 1/sqrt(#pixels)), additive Gaussian noise, noise scaled by the crop
displacement ("noise w.r.t. distance"), interpolation towards samples of the other labels ("line among
labels"), the 6-vs-8 binary subset, random down-sampling and the ``aug_data_set`` expander.  These run in
the DataLoader's worker processes (``DataLoader(..., transform=..., num_workers=N)``).
"""
from __future__ import annotations

import numpy as np


def _as_images(x):
    if x.ndim == 2:                       # flat rows: square single-channel images
        side = int(round(np.sqrt(x.shape[1])))
        return x.reshape(len(x), 1, side, side), True
    return x, False


def random_crop(batch, crop_hw, padding=0, rng=None, return_offsets=False):
    """Zero-pad by ``padding`` on each side, then crop ``crop_hw`` at a random offset per image."""
    rng = rng or np.random
    x, flat = _as_images(np.asarray(batch))
    n, c, h, w = x.shape
    if padding:
        x = np.pad(x, ((0, 0), (0, 0), (padding, padding), (padding, padding)))
    ch, cw = crop_hw
    oh = rng.randint(0, x.shape[2] - ch + 1, n)
    ow = rng.randint(0, x.shape[3] - cw + 1, n)
    rows = oh[:, None] + np.arange(ch)[None, :]                  # n x ch
    cols = ow[:, None] + np.arange(cw)[None, :]                  # n x cw
    out = x[np.arange(n)[:, None, None, None], np.arange(c)[None, :, None, None],
            rows[:, None, :, None], cols[:, None, None, :]]
    if flat:
        out = out.reshape(n, -1)
    return (out, oh - padding, ow - padding) if return_offsets else out


def random_crop_and_flip(batch, padding=2, rng=None):
    """CIFAR training distortion: padded random crop back to the input size + random horizontal flip."""
    rng = rng or np.random
    x = np.asarray(batch)
    out = random_crop(x, x.shape[-2:], padding, rng)
    flip = rng.rand(len(out)) < 0.5
    out[flip] = out[flip][..., ::-1]
    return out


def whiten(batch):
    """Per-image whitening: (x - mean) / max(std, 1 / sqrt(#values))."""
    x = np.asarray(batch, dtype=np.float32)
    flat = x.reshape(len(x), -1)
    mean = flat.mean(1, keepdims=True)
    std = np.maximum(flat.std(1, keepdims=True), 1.0 / np.sqrt(flat.shape[1]))
    return ((flat - mean) / std).reshape(x.shape).astype(np.float32)


def add_gaussian_noise(batch, mean=0.0, var=0.01, rng=None):
    rng = rng or np.random
    x = np.asarray(batch, dtype=np.float32)
    return (x + rng.normal(mean, np.sqrt(var), x.shape)).astype(np.float32)


def add_noise_wrt_distance(batch, crop_hw, padding=2, rng=None):
    """Random crop, then Gaussian noise whose std grows with how far each crop moved the image (the
    displacement norms are normalised over the batch)."""
    rng = rng or np.random
    x = np.asarray(batch, dtype=np.float32)
    out, oh, ow = random_crop(x, crop_hw, padding, rng, return_offsets=True)
    d = np.sqrt(oh.astype(np.float32) ** 2 + ow.astype(np.float32) ** 2)
    std = d / max(float(np.linalg.norm(d)), 1e-12)
    return (out + rng.normal(0.0, 1.0, out.shape) * std.reshape((-1,) + (1,) * (out.ndim - 1))).astype(np.float32)


def line_among_labels(data, labels, num_per_label=1, fraction=0.1, rng=None):
    """For every sample and every OTHER label: ``num_per_label`` new points on the line towards random
    samples of that label, x' = (1 - e) x + e o with e = fraction * |x| / |o|; labels are kept."""
    rng = rng or np.random
    data, labels = np.asarray(data, dtype=np.float32), np.asarray(labels)
    by_label = {k: data[labels == k] for k in np.unique(labels)}
    out_x, out_y = [], []
    norms = np.linalg.norm(data.reshape(len(data), -1), axis=1)
    for k, pool in by_label.items():
        if not len(pool):
            continue
        others = np.nonzero(labels != k)[0]
        if not len(others):
            continue
        pick = pool[rng.randint(0, len(pool), (len(others), num_per_label))]          # n_o x p x ...
        pn = np.linalg.norm(pick.reshape(len(others), num_per_label, -1), axis=2)
        eps = fraction * norms[others][:, None] / np.maximum(pn, 1e-12)
        eps = eps.reshape(eps.shape + (1,) * (data.ndim - 1))
        x = data[others][:, None]
        out_x.append(((1 - eps) * x + eps * pick).reshape((-1,) + data.shape[1:]))
        out_y.append(np.repeat(labels[others], num_per_label))
    return np.concatenate(out_x).astype(np.float32), np.concatenate(out_y)


def extract_binary(train_x, train_y, test_x, test_y, classes=(6, 8)):
    """The 6-vs-8 subset of a labelled split (mnist.py extract_for_binary)."""
    tr = np.isin(train_y, classes)
    te = np.isin(test_y, classes)
    return train_x[tr], train_y[tr], test_x[te], test_y[te]


def down_sample(data, labels, n, rng=None):
    rng = rng or np.random
    idx = rng.randint(0, len(data), n)
    return data[idx], labels[idx]


def aug_data_set(data, labels, times_expand=1, aug_type="crop", crop_hw=None, padding=2, rng=None):
    """Concatenate ``times_expand`` augmented copies: crop | noise | line_among_labels | fake (identity)."""
    rng = rng or np.random
    data = np.asarray(data, dtype=np.float32)
    xs, ys = [], []
    for _ in range(times_expand):
        if aug_type == "crop":
            x = random_crop(data, crop_hw or _as_images(data)[0].shape[-2:], padding, rng)
            y = labels
        elif aug_type == "noise":
            x, y = add_gaussian_noise(data, 0.0, 0.01, rng), labels
        elif aug_type == "line_among_labels":
            x, y = line_among_labels(data, labels, 1, 0.15, rng)
        elif aug_type == "fake":
            x, y = data, labels
        else:
            raise ValueError(aug_type)
        xs.append(x)
        ys.append(np.asarray(y))
    return np.concatenate(xs), np.concatenate(ys)
