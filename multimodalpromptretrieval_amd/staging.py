"""Host -> device image copies.

main.py's DataLoader yields batches whose images sit in pageable host memory (main.py:94-96, no
pin_memory); the reference copies them with ``.to(self.device)`` at
dataset/VQAFeatureDataset.py:189 and architectures/T5VisionModel.py:156.  (A worker-thread
uploader through a pinned ring was measured and dropped in round 3: the serving loop did not move,
3,915 / 3,992 vs 3,997 / 3,932 QA pairs/s, profiles/r03_hostab.txt.)
"""
from __future__ import annotations

import torch


def to_device(img, device, stream=None):
    """``img.to(device, float32)`` on the current stream (device tensors are only converted)."""
    return img.to(device, torch.float32, non_blocking=True)
