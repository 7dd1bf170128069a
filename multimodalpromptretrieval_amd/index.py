"""Device retrieval index: exhaustive L2 / cosine scan with fused top-k (libmpr.so).

Replaces the scan of dataset/VQAFeatureDataset.py:192-197
(``torch.cdist(combined, self.retrieval_embeddings)`` + ``torch.argsort(...)[:, s:s+k]``)
and backs the cosine surface of utils.py:57-62.
"""
from __future__ import annotations

import torch

from . import _lib

L2, COSINE = 0, 1


class DeviceIndex:
    """Index rows [n, d] fp32 resident in HBM (one shard: global ids start at ``row_offset``)."""

    def __init__(self, rows: torch.Tensor, device, metric: int = L2, row_offset: int = 0):
        _lib.ensure_device(device)
        self.device = torch.device(device)
        rows = rows.detach().to(torch.float32).contiguous()
        if rows.device.type == "cuda":
            # mpr_index_create copies with a synchronous copy on the legacy stream, which is not
            # ordered behind torch's (possibly non-blocking) current stream: let the rows land
            torch.cuda.current_stream(rows.device).synchronize()
        if rows.dim() != 2 or rows.shape[0] < 1:
            raise ValueError(f"index rows must be [n, d] with n >= 1, got {tuple(rows.shape)}")
        self.n, self.d = rows.shape
        self.metric = metric
        self.row_offset = row_offset
        h = _lib.ctypes.c_void_p()
        _lib.call("mpr_index_create", _lib.ptr(rows), self.n, self.d, metric, row_offset,
                  _lib.ctypes.byref(h))
        self._h = h

    def close(self):
        if getattr(self, "_h", None) is not None and _lib._lib is not None:
            _lib.load().mpr_index_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _q(self, q: torch.Tensor) -> torch.Tensor:
        q = q.to(self.device, torch.float32).contiguous()
        if q.dim() != 2 or q.shape[1] != self.d:
            raise ValueError(f"queries must be [b, {self.d}], got {tuple(q.shape)}")
        return q

    def search(self, q: torch.Tensor, k: int):
        """Best k rows per query: (dist fp32 [b, k], ids int64 [b, k]) on device.

        L2: ascending Euclidean distance (cdist); cosine: descending similarity; exact ties by
        lowest global id."""
        q = self._q(q)
        b = q.shape[0]
        ids = torch.empty((b, k), device=self.device, dtype=torch.int64)
        dist = torch.empty((b, k), device=self.device, dtype=torch.float32)
        _lib.call("mpr_index_search", self._h, _lib.ptr(q), b, int(k), _lib.ptr(ids),
                  _lib.ptr(dist), _lib.stream_ptr(self.device))
        return dist, ids

    def coarse_fallbacks(self) -> int:
        """Queries of the last search (current stream) that the coarse large-batch path handed to
        its exact fallback; -1 when that search did not take the coarse path.  Synchronises."""
        c = _lib.c_int32()
        _lib.call("mpr_index_coarse_fallbacks", self._h, _lib.stream_ptr(self.device),
                  _lib.ctypes.byref(c))
        return c.value

    def scores(self, q: torch.Tensor) -> torch.Tensor:
        """Full [b, n] distance (L2) or similarity (cosine) matrix (torch.cdist drop-in)."""
        q = self._q(q)
        out = torch.empty((q.shape[0], self.n), device=self.device, dtype=torch.float32)
        _lib.call("mpr_index_scores", self._h, _lib.ptr(q), q.shape[0], _lib.ptr(out),
                  _lib.stream_ptr(self.device))
        return out


def topk_merge(cand_dist: torch.Tensor, cand_ids: torch.Tensor, k: int, metric: int = L2):
    """Best k of per-shard candidates [b, n_cand] (same order/tie rule as DeviceIndex.search)."""
    cd = cand_dist.to(torch.float32).contiguous()
    ci = cand_ids.to(torch.int64).contiguous()
    b, n = cd.shape
    od = torch.empty((b, k), device=cd.device, dtype=torch.float32)
    oi = torch.empty((b, k), device=cd.device, dtype=torch.int64)
    _lib.call("mpr_topk_merge", _lib.ptr(cd), _lib.ptr(ci), b, n, int(k), metric, _lib.ptr(od),
              _lib.ptr(oi), _lib.stream_ptr(cd.device))
    return od, oi
