"""ctypes binding of libmpr.so (include/mpr.h).

The product path has no CPU fallback: importing a module that needs the library raises when the
shared object is missing or cannot be loaded, and every call raises ``RuntimeError`` with the
library's message on a non-zero return code.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_float, c_int32, c_int64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MPR_LIB", os.path.join(_HERE, "libmpr.so"))

F32P = POINTER(c_float)
I32P = POINTER(c_int32)
I64P = POINTER(c_int64)

# (name, restype, argtypes) — mirrors include/mpr.h one to one.
SIGNATURES = [
    ("mpr_init", c_int32, [c_int32]),
    ("mpr_last_error", ctypes.c_char_p, []),
    ("mpr_abi_version", c_int32, []),
    ("mpr_stream_sync", c_int32, [c_void_p]),
    ("mpr_index_create", c_int32, [c_void_p, c_int64, c_int32, c_int32, c_int64,
                                   POINTER(c_void_p)]),
    ("mpr_index_destroy", c_int32, [c_void_p]),
    ("mpr_index_rows", c_int64, [c_void_p]),
    ("mpr_index_search", c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_void_p,
                                   c_void_p]),
    ("mpr_index_scores", c_int32, [c_void_p, c_void_p, c_int32, c_void_p, c_void_p]),
    ("mpr_topk_merge", c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_int32, c_int32,
                                 c_void_p, c_void_p, c_void_p]),
    ("mpr_cosine_rows", c_int32, [c_void_p, c_void_p, c_int64, c_int32, c_float, c_void_p,
                                  c_void_p]),
    ("mpr_vit_create", c_int32, [I32P, c_int32, POINTER(c_void_p), c_int32, POINTER(c_void_p)]),
    ("mpr_vit_forward", c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_int64,
                                  c_void_p]),
    ("mpr_vit_forward_pair", c_int32, [c_void_p, c_int32, c_void_p, c_int64, c_void_p, c_int32,
                                       c_void_p, c_int64, c_void_p, c_int32, c_void_p]),
    ("mpr_clip_text_create", c_int32, [I32P, c_int32, POINTER(c_void_p), c_int32,
                                       POINTER(c_void_p)]),
    ("mpr_clip_text_forward", c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_int64,
                                        c_void_p]),
    ("mpr_t5_create", c_int32, [I32P, c_int32, POINTER(c_void_p), c_int32, I32P, I32P, c_int32,
                                POINTER(c_void_p)]),
    ("mpr_t5_embed", c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_int64, c_int32,
                               c_void_p]),
    ("mpr_t5_encode", c_int32, [c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_void_p,
                                c_void_p]),
    ("mpr_t5_generate", c_int32, [c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_int32,
                                  c_int32, c_int32, c_int32, c_void_p, c_void_p]),
    ("mpr_t5_logits", c_int32, [c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_void_p,
                                c_int32, c_void_p, c_void_p]),
    ("mpr_cross_entropy", c_int32, [c_void_p, c_void_p, c_int64, c_int32, c_void_p, c_void_p]),
    ("mpr_model_destroy", c_int32, [c_void_p]),
    ("mpr_probe_enable", c_int32, [c_int32]),
    ("mpr_probe_read", c_int32, [POINTER(ctypes.c_double), I64P, POINTER(ctypes.c_double),
                                 POINTER(ctypes.c_double)]),
]


def probe_enable(kind: int) -> None:
    call("mpr_probe_enable", kind)


def probe_read():
    """(kernel ms, launches, algorithmic flops, algorithmic bytes) since the last read."""
    ms, n, fl, by = ctypes.c_double(), c_int64(), ctypes.c_double(), ctypes.c_double()
    call("mpr_probe_read", ctypes.byref(ms), ctypes.byref(n), ctypes.byref(fl), ctypes.byref(by))
    return ms.value, n.value, fl.value, by.value

_lib = None


def load() -> ctypes.CDLL:
    """Load libmpr.so once; raise (never fall back) when it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"libmpr.so not found at {LIB_PATH}: build it with `python -c 'import "
            f"__graft_entry__ as g; g.build()'` (the product path has no CPU fallback)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def exported_symbols() -> list:
    return [name for name, _, _ in SIGNATURES]


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = load().mpr_last_error()
        raise RuntimeError(f"libmpr {what} failed ({rc}): {msg.decode() if msg else ''}")


def call(name: str, *args) -> int:
    rc = getattr(load(), name)(*args)
    check(rc, name)
    return rc


def ptr(t) -> c_void_p:
    """Device/host pointer of a torch tensor (must be contiguous where the ABI expects it)."""
    return c_void_p(t.data_ptr()) if t is not None else c_void_p(0)


def stream_ptr(device=None) -> c_void_p:
    import torch
    return c_void_p(torch.cuda.current_stream(device).cuda_stream)


_inited = set()


def ensure_device(device) -> None:
    """mpr_init(device index) once per device; the library then uses the current HIP device."""
    import torch
    dev = torch.device(device)
    if dev.type != "cuda":
        raise RuntimeError(f"libmpr runs on a GPU (cuda/HIP) device, got {dev}")
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    if idx not in _inited:
        call("mpr_init", c_int32(idx))
        _inited.add(idx)


def tensor_array(tensors) -> ctypes.Array:
    arr = (c_void_p * len(tensors))()
    for i, t in enumerate(tensors):
        arr[i] = t.data_ptr()
    return arr


def int_array(vals, ctype=c_int32) -> ctypes.Array:
    arr = (ctype * len(vals))()
    for i, v in enumerate(vals):
        arr[i] = int(v)
    return arr
