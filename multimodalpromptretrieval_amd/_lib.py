"""ctypes binding of libmpr.so (include/mpr.h).

The product path has no CPU fallback: importing a module that needs the library raises when the
shared object is missing or cannot be loaded, and every call raises ``RuntimeError`` with the
library's message on a non-zero return code.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_float, c_int32, c_int64, c_void_p  # noqa: F401

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
    ("mpr_stream_create", c_int32, [c_int32, POINTER(ctypes.c_uint32), c_int32,
                                    POINTER(c_void_p)]),
    ("mpr_stream_destroy", c_int32, [c_void_p]),
    ("mpr_index_create", c_int32, [c_void_p, c_int64, c_int32, c_int32, c_int64,
                                   POINTER(c_void_p)]),
    ("mpr_index_destroy", c_int32, [c_void_p]),
    ("mpr_index_rows", c_int64, [c_void_p]),
    ("mpr_index_search", c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_void_p,
                                   c_void_p]),
    ("mpr_index_scores", c_int32, [c_void_p, c_void_p, c_int32, c_void_p, c_void_p]),
    ("mpr_index_coarse_fallbacks", c_int32, [c_void_p, c_void_p, I32P]),
    ("mpr_topk_merge", c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_int32, c_int32,
                                 c_void_p, c_void_p, c_void_p]),
    ("mpr_topk_pack", c_int32, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
    ("mpr_topk_merge_packed", c_int32, [c_void_p, c_int32, c_int32, c_int32, c_int32, c_int32,
                                        c_int32, c_void_p, c_void_p, c_void_p]),
    ("mpr_sharded_search_all", c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_void_p,
                                         c_int32, c_int32, c_void_p, c_int32, c_void_p, c_void_p,
                                         c_void_p]),
    ("mpr_cosine_rows", c_int32, [c_void_p, c_void_p, c_int64, c_int32, c_float, c_void_p,
                                  c_void_p]),
    ("mpr_vit_create", c_int32, [I32P, c_int32, POINTER(c_void_p), c_int32, POINTER(c_void_p)]),
    ("mpr_vit_forward", c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_int64,
                                  c_void_p]),
    ("mpr_vit_forward_pair", c_int32, [c_void_p, c_int32, c_void_p, c_int64, c_void_p, c_int32,
                                       c_void_p, c_int64, c_void_p, c_int32, c_void_p]),
    ("mpr_encode_towers", c_int32, [c_void_p, c_int32, c_void_p, c_int64, c_void_p, c_int32,
                                    c_void_p, c_int64, c_void_p, c_int32, c_void_p, c_void_p,
                                    c_int32, c_int32, c_void_p, c_int64, c_int32, c_void_p]),
    ("mpr_encode_towers_multi", c_int32, [c_void_p, c_int32, c_void_p, c_int64, c_void_p,
                                          c_int32, c_void_p, c_int64, c_void_p, c_int32,
                                          c_void_p, c_int32, POINTER(c_void_p), I32P, I32P,
                                          POINTER(c_void_p), I64P, c_int32, c_void_p]),
    ("mpr_clip_text_create", c_int32, [I32P, c_int32, POINTER(c_void_p), c_int32,
                                       POINTER(c_void_p)]),
    ("mpr_clip_text_forward", c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_int64,
                                        c_void_p]),
    ("mpr_t5_create", c_int32, [I32P, c_int32, POINTER(c_void_p), c_int32, I32P, I32P, c_int32,
                                POINTER(c_void_p)]),
    ("mpr_t5_update", c_int32, [c_void_p, POINTER(c_void_p), c_int32, I32P, I32P]),
    ("mpr_t5_update_async", c_int32, [c_void_p, POINTER(c_void_p), c_int32, c_void_p]),
    ("mpr_t5_embed", c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_int64, c_int32,
                               c_void_p]),
    ("mpr_t5_encode", c_int32, [c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_void_p,
                                c_void_p]),
    ("mpr_t5_generate", c_int32, [c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_int32,
                                  c_int32, c_int32, c_int32, c_void_p, c_void_p]),
    ("mpr_t5_generate_slot", c_int32, [c_void_p, c_int32, c_void_p, c_void_p, c_int32, c_int32,
                                       c_int32, c_int32, c_int32, c_int32, c_void_p, c_void_p]),
    ("mpr_t5_generate_stop", c_int32, [c_void_p, c_int32, c_void_p, c_void_p, c_int32, c_int32,
                                       c_int32, c_int32, c_int32, c_int32, c_int32, c_void_p,
                                       POINTER(c_int32), c_void_p]),
    ("mpr_t5_generate_pair", c_int32, [c_void_p, c_int32, c_void_p, c_void_p, c_int32, c_int32,
                                       c_void_p, c_void_p, c_int32, c_int32, c_int32, c_int32,
                                       c_int32, c_int32, c_void_p, c_void_p, c_void_p]),
    ("mpr_t5_generate_batches", c_int32, [c_void_p, c_int32, c_int32, POINTER(c_void_p),
                                          POINTER(c_void_p), I32P, I32P, c_int32, c_int32,
                                          c_int32, c_int32, POINTER(c_void_p), c_void_p]),
    ("mpr_t5_generate_begin", c_int32, [c_void_p, c_int32, c_int32, POINTER(c_void_p),
                                        POINTER(c_void_p), I32P, I32P, c_int32, c_int32,
                                        c_int32, c_int32, c_int32, c_int32, POINTER(c_void_p),
                                        c_void_p]),
    ("mpr_t5_generate_poll", c_int32, [c_void_p, c_int32, c_int32, POINTER(c_int32),
                                       POINTER(c_int32), c_void_p]),
    ("mpr_t5_set_decode_stream", c_int32, [c_void_p, c_int32, c_void_p]),
    ("mpr_t5_logits", c_int32, [c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_void_p,
                                c_int32, c_void_p, c_void_p]),
    ("mpr_cross_entropy", c_int32, [c_void_p, c_void_p, c_int64, c_int32, c_void_p, c_void_p]),
    ("mpr_model_destroy", c_int32, [c_void_p]),
    ("mpr_probe_enable", c_int32, [c_int32]),
    ("mpr_probe_read", c_int32, [POINTER(ctypes.c_double), I64P, POINTER(ctypes.c_double),
                                 POINTER(ctypes.c_double)]),
    ("mpr_probe_replay", c_int32, [c_int32, c_void_p, POINTER(ctypes.c_double), I64P,
                                   POINTER(ctypes.c_double), POINTER(ctypes.c_double)]),
    ("mpr_probe_clear", c_int32, []),
    ("mpr_rccl_available", c_int32, [I32P]),
    ("mpr_debug_flags", c_int32, [I32P]),
    ("mpr_debug_check_guards", c_int32, [I32P, ctypes.c_char_p, c_int32]),
    ("mpr_debug_hash_buffers", c_int32, [POINTER(ctypes.c_uint64), POINTER(ctypes.c_uint64),
                                         I64P, c_int32, I32P]),
    ("mpr_debug_t5_workspace", c_int32, [c_void_p, c_int32, POINTER(ctypes.c_uint64), I64P,
                                         c_int32, I32P]),
    ("mpr_debug_t5_trace", c_int32, [c_void_p, c_int32, c_void_p, c_int64, I64P, I64P, c_int32,
                                     I32P, c_void_p]),
    ("mpr_gemm_f32", c_int32, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_int32,
                               c_int32, c_int32, c_void_p, c_int64, c_int32, c_void_p]),
    ("mpr_gemm_f32_many", c_int32, [c_int32, c_void_p, c_void_p]),
    ("mpr_t5_trainer_create", c_int32, [I32P, c_int32, I32P, I32P, c_int32, POINTER(c_void_p)]),
    ("mpr_t5_train_forward", c_int32, [c_void_p, POINTER(c_void_p), c_int32, c_void_p, c_void_p,
                                       c_int32, c_int32, c_void_p, c_void_p, c_int32, c_float,
                                       ctypes.c_uint64, ctypes.c_uint32, c_float, c_void_p,
                                       POINTER(c_int32), c_void_p]),
    ("mpr_t5_train_backward", c_int32, [c_void_p, c_int32, POINTER(c_void_p), c_int32, c_void_p,
                                        c_float, c_void_p, c_void_p, c_void_p, c_int32,
                                        POINTER(c_void_p), c_void_p, c_void_p]),
    ("mpr_t5_train_release", c_int32, [c_void_p, c_int32]),
    ("mpr_t5_trainer_trim", c_int32, [c_void_p, c_int32, c_void_p]),
    ("mpr_gemm_f32_splitk", c_int32, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64,
                                      c_int32, c_int32, c_int32, c_void_p, c_int64, c_int32,
                                      c_int32, c_void_p, c_void_p]),
    ("mpr_pack_x3_bytes", c_int32, [c_int64, c_int64, I64P]),
    ("mpr_pack_x3", c_int32, [c_void_p, c_int64, c_int64, c_int64, c_void_p, c_int64, c_void_p]),
    ("mpr_gemm_f32_packed", c_int32, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p,
                                      c_int64, c_int32, c_int32, c_int32, c_void_p, c_int64,
                                      c_int32, c_void_p]),
    ("mpr_transpose", c_int32, [c_void_p, c_int64, c_int64, c_int64, c_void_p, c_int64,
                                c_void_p]),
    ("mpr_rmsnorm_fwd", c_int32, [c_void_p, c_int32, c_int32, c_void_p, c_float, c_float,
                                  c_void_p, c_void_p, c_void_p]),
    ("mpr_rmsnorm_bwd", c_int32, [c_void_p, c_int32, c_int32, c_void_p, c_void_p, c_void_p,
                                  c_float, c_void_p, c_int32, c_void_p, c_void_p, c_void_p]),
    ("mpr_attn_train_fwd", c_int32, [c_void_p, c_int64, c_int64, c_void_p, c_int64, c_int64,
                                     c_void_p, c_int64, c_int64, c_int32, c_int32, c_int32,
                                     c_int32, c_int32, c_void_p, c_void_p, c_int32, c_void_p,
                                     c_int64, c_int64, c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                     ctypes.c_uint32, c_float, c_void_p]),
    ("mpr_attn_train_bwd", c_int32, [c_void_p, c_int64, c_int64, c_void_p, c_int64, c_int64,
                                     c_void_p, c_int64, c_int64, c_int32, c_int32, c_int32,
                                     c_int32, c_void_p, c_void_p, c_int64, c_int64, c_void_p,
                                     c_void_p, c_int64, c_int64, c_void_p, c_int64, c_int64,
                                     c_void_p, c_int64, c_int64, c_void_p, c_int32,
                                     ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, c_float,
                                     c_void_p]),
    ("mpr_dropout", c_int32, [c_void_p, c_int64, ctypes.c_uint64, ctypes.c_uint32,
                              ctypes.c_uint32, c_float, c_void_p, c_void_p, c_void_p]),
    ("mpr_rel_gather", c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_void_p]),
    ("mpr_rel_scatter", c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_int32, c_void_p,
                                  c_void_p]),
    ("mpr_relu_bwd", c_int32, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
    ("mpr_add", c_int32, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
    ("mpr_ce_train", c_int32, [c_void_p, c_int64, c_int32, c_void_p, c_float, c_float, c_void_p,
                               c_void_p, c_void_p, c_void_p, c_int64, c_void_p]),
    ("mpr_gather_rows", c_int32, [c_void_p, c_void_p, c_int64, c_int32, c_void_p, c_void_p]),
    ("mpr_embed_bwd", c_int32, [c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_int32,
                                c_void_p, c_void_p]),
    ("mpr_dot_reduce", c_int32, [c_void_p, c_void_p, c_int32, I64P, I64P, I64P, c_int64,
                                 c_int64, c_int64, c_int32, c_void_p, c_void_p]),
    ("mpr_cos_combine", c_int32, [c_void_p, c_void_p, c_void_p, c_int32, I64P, I64P, I64P, I64P,
                                  c_float, c_void_p, c_void_p]),
]


def probe_enable(kind: int) -> None:
    call("mpr_probe_enable", kind)


def probe_read():
    """(kernel ms, launches, algorithmic flops, algorithmic bytes) since the last read."""
    ms, n, fl, by = ctypes.c_double(), c_int64(), ctypes.c_double(), ctypes.c_double()
    call("mpr_probe_read", ctypes.byref(ms), ctypes.byref(n), ctypes.byref(fl), ctypes.byref(by))
    return ms.value, n.value, fl.value, by.value

def probe_replay(iters: int = 1, device=None):
    """Replay the GEMM launches recorded under probe_enable(3) back to back on the current
    stream: (kernel ms, launches, algorithmic flops, algorithmic bytes)."""
    ms, n, fl, by = ctypes.c_double(), c_int64(), ctypes.c_double(), ctypes.c_double()
    call("mpr_probe_replay", int(iters), stream_ptr(device), ctypes.byref(ms), ctypes.byref(n),
         ctypes.byref(fl), ctypes.byref(by))
    return ms.value, n.value, fl.value, by.value


def probe_clear() -> None:
    call("mpr_probe_clear")


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


def to_device_async(t, device, dtype=None):
    """Host tensor -> device on the current stream without blocking the host: staged through
    pinned memory (a pageable source makes the copy wait, on the host, for all earlier work on
    the stream — and, with more streams than the 4 hardware queues, for work of other streams
    that share its queue).  Device tensors are only converted."""
    import torch
    if t.device.type != "cpu" or os.environ.get("MPR_PIN_H2D") == "0":
        return t.to(device, dtype) if dtype is not None else t.to(device)
    if dtype is not None:
        t = t.to(dtype)
    return t.contiguous().pin_memory().to(device, non_blocking=True)


def stream_ptr(device=None) -> c_void_p:
    import torch
    return c_void_p(torch.cuda.current_stream(device).cuda_stream)


_inited = set()
_role_streams = {}


def _cu_count(idx: int) -> int:
    import torch
    return torch.cuda.get_device_properties(idx).multi_processor_count


def decode_cus(idx: int) -> int:
    """CUs reserved for the T5 decode chain (MPR_DECODE_CUS; default 0 = no partition).
    Measured on MI355X (bench c2): 32 / 64 / 96 reserved CUs ran 805 / 858 / 838 QA pairs/s
    against 1362 unpartitioned — the decode launches (up to 1004 blocks for the lm_head) need the
    whole chip, so the partition is off by default."""
    n = int(os.environ.get("MPR_DECODE_CUS", "0"))
    total = _cu_count(idx)
    return n if 0 < n < total else 0


def stream_priorities() -> tuple:
    """(retrieval-encoder streams, generate streams) priorities, MPR_STREAM_PRIO = "enc"
    (the retrieval encoders first — the host waits on their result to build prompts),
    "gen" (default: the generate streams first — with the towers back to back, the pair
    decodes, a chain of ~1000 small launches, are the co-critical path; gen / both / enc / none
    = 2633 / 2606 / 2590 / 2548 QA pairs/s), "both" or "none".  Lower is higher (-1 = high).
    Leaving CUs to the generate streams through a CU mask on the encoder streams measured far
    slower (8 / 16 / 32 CUs: 1251 / 1039 / 1391)."""
    mode = os.environ.get("MPR_STREAM_PRIO", "gen")
    return {"enc": (-1, 0), "gen": (0, -1), "both": (-1, -1)}.get(mode, (0, 0))


def separate_decode_stream(idx: int) -> bool:
    """The decode loop gets a stream of its own only with a CU partition."""
    return bool(decode_cus(idx))


# Created eagerly in this order (ensure_device).  The index build's second tower slot is made
# second: created on first use it landed beside the first slot and the build ran at 8,530-9,040
# rows/s against 10,470-11,300 with it here; training and serving unchanged (same-box A/Bs,
# profiles/r06_stream_roles.txt).
PIPELINE_ROLES = ("encode:towers", "encode:towers1", "train:spec", "gen:0", "gen:1")


def role_stream(device, role: str):
    """A process-lifetime stream for one role of the serving pipeline: ``"decode"`` (the T5
    greedy loop, CU partition only), ``"gen:<slot>"`` (a batch's T5 generate in the serving loop)
    or ``"encode:<tag>"`` (retrieval towers).  With a CU partition
    (decode_cus() > 0) the decode stream is restricted to the first n CUs (mask bits [0, n)) and
    the encoder streams to the rest; ``"train:spec"`` is the trainer's speculative backward
    (encoder priority); otherwise plain non-blocking streams with
    stream_priorities().  Returned as torch.cuda.ExternalStream so torch work can be enqueued on
    it as well."""
    import torch
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    key = (idx, role)
    st = _role_streams.get(key)
    if st is not None:
        return st
    ensure_device(dev)
    n = decode_cus(idx)
    total = _cu_count(idx)
    words = (total + 31) // 32
    h = c_void_p()
    with torch.cuda.device(idx):
        if n:
            bits = range(0, n) if role == "decode" else range(n, total)
            mask = (ctypes.c_uint32 * words)()
            for b in bits:
                mask[b // 32] |= 1 << (b % 32)
            call("mpr_stream_create", 0, mask, words, ctypes.byref(h))
        else:
            pe, pg = stream_priorities()
            call("mpr_stream_create", pe if role.startswith(("encode", "train")) else pg, None,
                 0, ctypes.byref(h))
    st = torch.cuda.ExternalStream(h.value, device=dev)
    _role_streams[key] = st
    return st


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
        # The pipeline's role streams are created once, in a fixed order, right after init
        # (MPR_EAGER_STREAMS=0: on first use instead).  A stream's hardware queue (4 per process)
        # is fixed at its creation; created on first use, their queue sharing depended on what
        # ran before (a training step after another model's serving loop: 24 ms against 13.5,
        # profiles/r05_train_streams.txt).  (Round 5 kept this opt-in because with it the serving
        # loop's answers changed more often; the cause was packed-FP32 results corrupted beside
        # other kernels' MFMA waves, fixed by building without packed FP32 ops)
        if os.environ.get("MPR_EAGER_STREAMS", "1") == "1":
            order = os.environ.get("MPR_EAGER_ORDER")  # A/B of the creation order
            for role in (order.split(",") if order else PIPELINE_ROLES):
                role_stream(torch.device("cuda", idx), role)


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
