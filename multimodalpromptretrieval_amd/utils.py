"""Drop-in for the similarity helper of the reference's utils.py.

``cosine_similarity`` (utils.py:57-62) is ``sum(x1*x2, dim) / clamp(|x1|*|x2|, eps)`` then
``squeeze()``, for any broadcastable pair, computed in libmpr on the GPU:
* aligned rows (``x1.shape == x2.shape``): the fused row kernel over ``dim``;
* pairwise (``x1 [B,1,D]`` vs ``x2 [1,N,D]`` with ``dim=2`` — the retrieval-matrix pattern, eps
  1e-8, D % 16 == 0): the index scan kernel in cosine mode;
* every other layout: the reference's three reductions as written — ``x1 . x2`` over the
  broadcast axis, ``norm(x1, 2, dim)`` and ``norm(x2, 2, dim)`` over each operand's own axis —
  then the clamped division broadcasting the three (mpr_dot_reduce, mpr_cos_combine).
Tensors on the host are computed on the current GPU and the result comes back to the host (the
reference's result lives where its inputs did); the result dtype is the inputs' promoted dtype.
Mixed devices and non-broadcastable shapes raise as torch does.  Without a GPU the call raises:
the product computes on the MI355X, there is no CPU path.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from .index import COSINE, DeviceIndex


def _i64(vals):
    return _lib.int_array(list(vals), ctypes.c_int64)


def _check_dim(dim: int, nd: int) -> int:
    lo, hi = (-nd, nd - 1) if nd > 0 else (-1, 0)
    if not lo <= dim <= hi:
        raise IndexError(f"Dimension out of range (expected to be in range of [{lo}, {hi}], "
                         f"but got {dim})")
    return dim % nd if nd > 0 else 0


def _dot(a: torch.Tensor, b: torch.Tensor, shape, axis: int, take_sqrt: bool) -> torch.Tensor:
    """sum_t a[.., t, ..] * b[.., t, ..] over `axis` of the broadcast `shape` (sqrt optional)."""
    ae, be = a.expand(shape), b.expand(shape)
    keep = [d for d in range(len(shape)) if d != axis]
    out_shape = [shape[d] for d in keep]
    out = torch.empty(out_shape, device=a.device, dtype=torch.float32)
    D = shape[axis] if len(shape) else 1
    ta = ae.stride(axis) if len(shape) else 0
    tb = be.stride(axis) if len(shape) else 0
    _lib.call("mpr_dot_reduce", _lib.ptr(ae), _lib.ptr(be), len(out_shape), _i64(out_shape),
              _i64([ae.stride(d) for d in keep]), _i64([be.stride(d) for d in keep]), D, ta, tb,
              1 if take_sqrt else 0, _lib.ptr(out), _lib.stream_ptr(a.device))
    return out


def _combine(w12: torch.Tensor, n1: torch.Tensor, n2: torch.Tensor, eps: float) -> torch.Tensor:
    shape = torch.broadcast_shapes(w12.shape, torch.broadcast_shapes(n1.shape, n2.shape))
    ops = [x.expand(shape) for x in (w12, n1, n2)]
    out = torch.empty(shape, device=w12.device, dtype=torch.float32)
    _lib.call("mpr_cos_combine", _lib.ptr(ops[0]), _lib.ptr(ops[1]), _lib.ptr(ops[2]),
              len(shape), _i64(shape), *[_i64(o.stride()) for o in ops], float(eps),
              _lib.ptr(out), _lib.stream_ptr(w12.device))
    return out


def _on_gpu(x1: torch.Tensor, x2: torch.Tensor):
    if x1.device != x2.device:
        raise RuntimeError(f"Expected all tensors to be on the same device, but found at least "
                           f"two devices, {x1.device} and {x2.device}!")
    if x1.device.type == "cuda":
        return x1.device
    if not torch.cuda.is_available():
        raise RuntimeError("cosine_similarity: libmpr computes on the GPU and none is available")
    return torch.device("cuda", torch.cuda.current_device())


def cosine_similarity(x1: torch.Tensor, x2: torch.Tensor, dim: int = 1, eps: float = 1e-8):
    home = x1.device
    dev = _on_gpu(x1, x2)
    out_dtype = torch.result_type(x1, x2)
    if not out_dtype.is_floating_point:
        out_dtype = torch.get_default_dtype()
    _lib.ensure_device(dev)
    a = x1.to(dev, torch.float32)
    b = x2.to(dev, torch.float32)
    shape = torch.broadcast_shapes(a.shape, b.shape)  # raises as x1 * x2 would
    nd = len(shape)
    axis = _check_dim(dim, nd)
    if a.shape == b.shape and nd > 0:
        ac = a.movedim(axis, -1).contiguous()
        bc = b.movedim(axis, -1).contiguous()
        out = torch.empty(ac.shape[:-1], device=dev, dtype=torch.float32)
        _lib.call("mpr_cosine_rows", _lib.ptr(ac), _lib.ptr(bc), out.numel(), ac.shape[-1],
                  float(eps), _lib.ptr(out), _lib.stream_ptr(dev))
    elif (nd == 3 and axis == 2 and a.dim() == 3 and b.dim() == 3 and a.shape[1] == 1
          and b.shape[0] == 1 and a.shape[2] == b.shape[2] and eps == 1e-8
          and a.shape[2] % 16 == 0 and b.shape[1] > 0):
        ix = DeviceIndex(b[0], dev, metric=COSINE)
        out = ix.scores(a[:, 0, :])
    else:
        w12 = _dot(a, b, shape, axis, take_sqrt=False)
        n1 = _dot(a, a, a.shape, _check_dim(dim, a.dim()), take_sqrt=True)
        n2 = _dot(b, b, b.shape, _check_dim(dim, b.dim()), take_sqrt=True)
        out = _combine(w12, n1, n2, eps)
    return out.squeeze().to(home, out_dtype)
