"""Oracle: the counter-based dropout masks of the device training step (TEST INFRASTRUCTURE ONLY).

numpy restatement of ``mpr_dropout`` / the attention kernels' probability dropout
(multimodalpromptretrieval_amd/csrc/train.hip ``drop_factor``): element e of site s under seed S
is kept iff the top 24 bits of splitmix64(S ^ s * 0x9E3779B97F4A7C15 + e * 0xD1B54A32D192ED03)
are >= thresh = int(p * 2^24); kept elements are multiplied by float32(1 / (1 - p)).  Used to
inject the same masks into the reference's T5 (transformers, train mode) at the sites
transformers applies dropout (tests/golden/make_goldens.py make_g12), whose gradients the device
step is then checked against (tests/test_gpu_train.py).
"""
from __future__ import annotations

import numpy as np
import torch

_M = np.uint64(0xFFFFFFFFFFFFFFFF)


def keep(seed: int, site: int, n: int, p: float) -> np.ndarray:
    """bool [n]: which of the n elements (row-major order) the mask keeps."""
    thresh = np.uint64(int(p * (1 << 24)))
    if thresh == 0:
        return np.ones(n, dtype=bool)
    with np.errstate(over="ignore"):
        x = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) ^ (np.uint64(site) * np.uint64(0x9E3779B97F4A7C15))
        x = x + np.arange(n, dtype=np.uint64) * np.uint64(0xD1B54A32D192ED03)
        x ^= x >> np.uint64(30)
        x *= np.uint64(0xBF58476D1CE4E5B9)
        x ^= x >> np.uint64(27)
        x *= np.uint64(0x94D049BB133111EB)
        x ^= x >> np.uint64(31)
    return (x >> np.uint64(40)) >= thresh


def factors(seed: int, site: int, shape, p: float) -> torch.Tensor:
    """float32 tensor of `shape`: 1/(1-p) where kept, 0 where dropped."""
    n = int(np.prod(shape))
    scale = np.float32(1.0 / (1.0 - p))
    f = np.where(keep(seed, site, n, p), scale, np.float32(0.0)).astype(np.float32)
    return torch.from_numpy(f.reshape(tuple(shape)))
