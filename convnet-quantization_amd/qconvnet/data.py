"""Synthetic CIFAR-shaped inputs: x = (U[0,1) - mean_c)/std_c,
fp32 NCHW, drawn from numpy PCG64 so every machine sees the same tensors.
Normalisation constants of /root/reference/utils/dataset_manager.py:41-44
(CIFAR-10) and :27 (ImageNet).  CIFAR-10 itself is not on disk and there is no
network, so benchmarks and default calibration use these tensors."""
from __future__ import annotations

import numpy as np
import torch

CIFAR_MEAN = (0.4914, 0.4822, 0.4465)
CIFAR_STD = (0.2023, 0.1994, 0.2010)
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def synthetic_images(n, seed, hw=32, mean=CIFAR_MEAN, std=CIFAR_STD):
    rng = np.random.Generator(np.random.PCG64(seed))
    u = rng.random((n, 3, hw, hw), dtype=np.float32)
    m = np.asarray(mean, np.float32).reshape(1, 3, 1, 1)
    s = np.asarray(std, np.float32).reshape(1, 3, 1, 1)
    return ((u - m) / s).astype(np.float32)


def _class_templates(hw=32, k=10, seed=1234):
    """k fixed smooth colour patterns (8x8 noise upsampled) — the class means
    of the synthetic task."""
    rng = np.random.Generator(np.random.PCG64(seed))
    low = rng.standard_normal((k, 3, 8, 8)).astype(np.float32)
    t = np.repeat(np.repeat(low, hw // 8, axis=2), hw // 8, axis=3)
    return t


def synthetic_task(n, seed, hw=32, noise=1.3):
    """A learnable 10-class CIFAR-shaped task (CIFAR-10 is not on disk):
    x = template[y] * contrast + smooth clutter + pixel noise, randomly
    flipped, squashed to [0,1] and CIFAR-normalised.  Returns (x, y) numpy."""
    rng = np.random.Generator(np.random.PCG64(seed))
    t = _class_templates(hw)
    y = rng.integers(0, 10, n)
    contrast = rng.uniform(0.5, 1.5, (n, 1, 1, 1)).astype(np.float32)
    clutter = np.repeat(np.repeat(rng.standard_normal((n, 3, hw // 4, hw // 4)).astype(np.float32),
                                  4, axis=2), 4, axis=3)
    x = t[y] * contrast + noise * clutter + 0.5 * rng.standard_normal((n, 3, hw, hw)).astype(np.float32)
    flip = rng.random(n) < 0.5
    x[flip] = x[flip][..., ::-1]
    u = 1.0 / (1.0 + np.exp(-0.7 * x))
    m = np.asarray(CIFAR_MEAN, np.float32).reshape(1, 3, 1, 1)
    s = np.asarray(CIFAR_STD, np.float32).reshape(1, 3, 1, 1)
    return ((u - m) / s).astype(np.float32), y.astype(np.int64)


def calibration_batches(loader=None, max_batches=None, default_images=512, default_seed=1):
    """Images from a reference-style loader ((images, labels) batches), a
    tensor, or — when None — the first 512 synthetic images of seed 1."""
    if loader is None:
        return [torch.from_numpy(synthetic_images(default_images, default_seed))]
    if torch.is_tensor(loader):
        return [loader]
    out = []
    for i, batch in enumerate(loader):
        if max_batches is not None and i >= max_batches:
            break
        out.append(batch[0] if isinstance(batch, (tuple, list)) else batch)
    return out


class SyntheticLoader:
    """A minimal DataLoader stand-in yielding (images, labels) like the
    reference's CIFAR-10 test loader (dataset_manager.py:130-166)."""

    def __init__(self, n=1024, batch_size=1024, seed=0, labels=None):
        self.x = torch.from_numpy(synthetic_images(n, seed))
        self.y = torch.zeros(n, dtype=torch.long) if labels is None else torch.as_tensor(labels)
        self.batch_size = batch_size

    def __iter__(self):
        for i in range(0, self.x.shape[0], self.batch_size):
            yield self.x[i:i + self.batch_size], self.y[i:i + self.batch_size]

    def __len__(self):
        return (self.x.shape[0] + self.batch_size - 1) // self.batch_size
