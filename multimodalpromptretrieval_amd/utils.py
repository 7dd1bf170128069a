"""Drop-in for the similarity helper of the reference's utils.py.

``cosine_similarity`` (utils.py:57-62) is ``sum(x1*x2, dim) / clamp(|x1|*|x2|, eps)`` then
``squeeze()``.  On a GPU tensor it runs in libmpr:
* aligned rows (``x1.shape == x2.shape``): row-wise kernel over ``dim``;
* pairwise (``x1 [B,1,D]`` vs ``x2 [1,N,D]`` with ``dim=2`` — the retrieval-matrix pattern): the
  index scan kernel in cosine mode.
Other layouts raise (no silent torch fallback on the product path).  CPU tensors are not
accepted either: the product computes on the MI355X.
"""
from __future__ import annotations

import torch

from . import _lib
from .index import COSINE, DeviceIndex


def cosine_similarity(x1: torch.Tensor, x2: torch.Tensor, dim: int = 1, eps: float = 1e-8):
    if x1.device.type != "cuda" or x2.device.type != "cuda":
        raise RuntimeError("cosine_similarity: libmpr computes on the GPU; pass cuda tensors")
    nd = x1.dim()
    dim = dim % nd
    if x1.shape == x2.shape:
        a = x1.movedim(dim, -1).to(torch.float32).contiguous()
        b = x2.movedim(dim, -1).to(torch.float32).contiguous()
        lead = a.shape[:-1]
        d = a.shape[-1]
        out = torch.empty(lead, device=a.device, dtype=torch.float32)
        m = out.numel()
        _lib.ensure_device(a.device)
        _lib.call("mpr_cosine_rows", _lib.ptr(a), _lib.ptr(b), m, d, float(eps), _lib.ptr(out),
                  _lib.stream_ptr(a.device))
        return out.squeeze()
    if (nd == 3 and dim == 2 and x1.shape[1] == 1 and x2.shape[0] == 1
            and x1.shape[2] == x2.shape[2]):
        q = x1[:, 0, :]
        rows = x2[0]
        if eps != 1e-8:
            raise NotImplementedError("pairwise cosine_similarity supports eps=1e-8 only")
        if rows.shape[1] % 16:
            raise NotImplementedError("pairwise cosine_similarity needs D % 16 == 0")
        ix = DeviceIndex(rows, rows.device, metric=COSINE)
        return ix.scores(q).squeeze()
    raise NotImplementedError(f"cosine_similarity: unsupported broadcast {tuple(x1.shape)} vs "
                              f"{tuple(x2.shape)} over dim {dim}")
