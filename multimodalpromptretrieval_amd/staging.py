"""Host -> device image copies off the host's critical path.

main.py's DataLoader yields batches whose images sit in pageable host memory (main.py:94-96, no
pin_memory); the reference copies them with ``.to(self.device)`` at
dataset/VQAFeatureDataset.py:189 and architectures/T5VisionModel.py:156.  A pageable copy makes
the calling thread wait — for the staging memcpy, and for earlier work on the stream it is
enqueued on — which in a serving loop is the thread that should be building the next batch's
prompts.  ``ImageUploader`` takes that copy off it: a worker thread copies the batch's image into
a pinned buffer of a small ring (CPU memcpy, the GIL released) and enqueues the DMA from it on a
copy stream (mode 1) or leaves the DMA to the consumer's stream (mode 2).  Results are the same
bytes; only who waits changes.  Off by default (``MPR_UPLOAD_THREAD``, ``ImageUploader.mode``).
"""
from __future__ import annotations

import os
import threading
from concurrent.futures import ThreadPoolExecutor

import torch


class ImageUploader:
    SLOTS = 6  # pinned staging buffers in flight (a serving loop stages ~2 passes ahead)

    def __init__(self, device):
        self.device = torch.device(device)
        self.dma_here = self.mode() == 1
        self.stream = torch.cuda.Stream(self.device) if self.dma_here else None
        self.pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="mpr-upload")
        self.pending = {}  # id(host image) -> (host image, future)
        # [pinned buffer, last DMA's event, released: the slot's last image was taken or dropped]
        self.ring = [[None, None, threading.Event()] for _ in range(self.SLOTS)]
        for r in self.ring:
            r[2].set()
        self.next = 0
        self.lock = threading.Lock()

    @staticmethod
    def mode() -> int:
        """MPR_UPLOAD_THREAD: 0 off (default: measured 3960-4060 vs 3340-3430 QA pairs/s with
        mode 1), 1 the worker copies into pinned memory and enqueues the DMA on its copy stream,
        2 the worker only copies into pinned memory; the DMA is enqueued by the consumer on its
        own stream (no extra stream)."""
        try:
            return int(os.environ.get("MPR_UPLOAD_THREAD", "0"))
        except ValueError:
            return 0

    @classmethod
    def enabled(cls) -> bool:
        return cls.mode() in (1, 2)

    def submit(self, img) -> None:
        """Start uploading a host image tensor (no-op for device tensors / already submitted)."""
        if not isinstance(img, torch.Tensor) or img.device.type != "cpu" or img.numel() == 0:
            return
        with self.lock:
            ent = self.pending.get(id(img))
            if ent is not None and ent[0] is img:
                return
            while len(self.pending) >= self.SLOTS:  # submitted but never taken: drop the oldest
                old = self.pending.pop(next(iter(self.pending)))
                self.ring[old[2]][2].set()
            slot = self.next
            self.next = (self.next + 1) % self.SLOTS
            self.ring[slot][2].wait()  # its previous image was taken (its DMA enqueued) or dropped
            self.ring[slot][2].clear()
            self.pending[id(img)] = (img, self.pool.submit(self._work, img, slot), slot)

    def _work(self, img, slot):
        buf, ev, _ = self.ring[slot]
        if ev is not None:
            ev.synchronize()  # the slot's previous DMA has read the buffer
        src = img.to(torch.float32) if img.dtype != torch.float32 else img
        src = src.contiguous()
        if buf is None or buf.numel() < src.numel():
            buf = torch.empty(src.numel(), dtype=torch.float32, pin_memory=True)
        pinned = buf[:src.numel()].view(src.shape)
        pinned.copy_(src)
        if not self.dma_here:  # mode 2: the consumer enqueues the DMA (take)
            self.ring[slot][0], self.ring[slot][1] = buf, None
            return pinned, slot
        with torch.cuda.device(self.device), torch.cuda.stream(self.stream):
            dev = torch.empty(src.shape, device=self.device, dtype=torch.float32)
            dev.copy_(pinned, non_blocking=True)
            done = torch.cuda.Event()
            done.record(self.stream)
        self.ring[slot][0], self.ring[slot][1] = buf, done
        return dev, done

    def take(self, img, stream=None):
        """The uploaded device copy of ``img``, ordered before later work on ``stream`` (default:
        the current stream), or None when it was not submitted."""
        with self.lock:
            ent = self.pending.pop(id(img), None)
        if ent is None or ent[0] is not img:
            return None
        stream = stream or torch.cuda.current_stream(self.device)
        if not self.dma_here:
            pinned, slot = ent[1].result()
            with torch.cuda.stream(stream):
                dev = torch.empty(pinned.shape, device=self.device, dtype=torch.float32)
                dev.copy_(pinned, non_blocking=True)
                done = torch.cuda.Event()
                done.record(stream)
            self.ring[slot][1] = done  # the slot is reusable once this DMA has read it
            self.ring[slot][2].set()
            return dev
        dev, done = ent[1].result()
        self.ring[ent[2]][2].set()
        stream.wait_event(done)
        dev.record_stream(stream)
        return dev


_UPLOADERS = {}


def uploader(device):
    """The process's ImageUploader for ``device`` (None when MPR_UPLOAD_THREAD=0)."""
    if not ImageUploader.enabled():
        return None
    dev = torch.device(device)
    key = (dev.type, dev.index)
    up = _UPLOADERS.get(key)
    if up is None:
        up = _UPLOADERS[key] = ImageUploader(dev)
    return up


def to_device(img, device, stream=None):
    """``img.to(device, float32)``: the uploader's copy when one was submitted, else a direct
    copy (device tensors are only converted)."""
    if isinstance(img, torch.Tensor) and img.device.type == "cpu":
        up = uploader(device) if _UPLOADERS else None
        if up is not None:
            dev = up.take(img, stream)
            if dev is not None:
                return dev
    return img.to(device, torch.float32, non_blocking=True)
