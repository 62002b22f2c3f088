"""Data layer.

* :class:`DataSet` — in-memory arrays with the reference's epoch-wrapping ``next_batch(bs)`` and fixed-seed
  reshuffle per epoch (pytorch_code/mnist/mnist.py:38-131, SEED=66478).
* :func:`read_mnist` — IDX files through the C++ reader, pixels normalised to [-0.5, 0.5]
  (mnist.py:143), NCHW 1x28x28 or flat 784 (PP-06 / TF-07), optional one-hot labels (mnist.py:205-215).
* :func:`read_cifar10` — CIFAR-10 *binary* batches (``data_batch_*.bin``), decoded with a proper
  channel transpose (the reference's ``reshape`` scrambles pixels, defect D10); the reference's pickled
  python batches are deliberately not read (unpickling files is unsafe).
* :class:`SyntheticDataset` — device-resident random tensors of any model's input shape (no network here:
  benchmarks and tests use synthetic data of the real shapes).
* :class:`DataLoader` — batches from any of the above with a background prefetch thread, pinned host
  memory and async host->device copies (the reference's custom multiprocess loader, PT-11
  my_data_loader.py:137-319, incl. ``next_batch``); ``skip(n)`` fast-forwards a resumed run without
  building the skipped batches.
* :class:`DeviceDataLoader` — the whole dataset in HBM, batches gathered on the device (synthetic data and
  small datasets; the CLI's ``--synthetic`` path on a GPU).
* :class:`MNISTDataset` / :class:`Cifar10Dataset` — torch ``Dataset`` wrappers (PT-12).
"""
from .datasets import (Cifar10Dataset, DataLoader, DataSet, DeviceDataLoader, MNISTDataset,  # noqa: F401
                       SyntheticDataset,
                       SyntheticTokens, augment_crop_flip, read_cifar10, read_mnist, write_mnist_like)
