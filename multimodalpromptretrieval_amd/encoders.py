"""Device CLIP encoders (ViT-B/32 image tower, text tower) backed by libmpr.so.

Replace the openai CLIP calls of the reference:
* ``clip_model.encode_image`` — dataset/VQAFeatureDataset.py:146,189 (mode "cls")
* ``vision_model.visual`` monkey-patched to ``get_image_token_features`` —
  architectures/T5VisionModel.py:46-48,112-139 (mode "tokens")
* ``clip_model.encode_text(clip.tokenize(q))`` — dataset/VQAFeatureDataset.py:147,190
Weights are openai-CLIP-named state-dict tensors; the library copies them into its own HBM
layout at construction (re-create the encoder to pick up new weights).
"""
from __future__ import annotations

import torch

from . import _lib

CLS, TOKENS = 0, 1


def _block_tensors(sd: dict, prefix: str, layers: int) -> list:
    out = []
    for i in range(layers):
        p = f"{prefix}.resblocks.{i}"
        out += [sd[p + ".ln_1.weight"], sd[p + ".ln_1.bias"], sd[p + ".attn.in_proj_weight"],
                sd[p + ".attn.in_proj_bias"], sd[p + ".attn.out_proj.weight"],
                sd[p + ".attn.out_proj.bias"], sd[p + ".ln_2.weight"], sd[p + ".ln_2.bias"],
                sd[p + ".mlp.c_fc.weight"], sd[p + ".mlp.c_fc.bias"],
                sd[p + ".mlp.c_proj.weight"], sd[p + ".mlp.c_proj.bias"]]
    return out


def _count_layers(sd: dict, prefix: str) -> int:
    n = 0
    while f"{prefix}.resblocks.{n}.ln_1.weight" in sd:
        n += 1
    return n


def _host_f32(ts: list) -> list:
    """fp32 contiguous tensors (host or device: the library copies with hipMemcpyDefault)."""
    return [t.detach().to(torch.float32).contiguous() for t in ts]


class _Handle:
    def __init__(self):
        self._h = None

    def close(self):
        if self._h is not None and _lib._lib is not None:
            _lib.load().mpr_model_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceViT(_Handle):
    """CLIP VisionTransformer (openai naming, prefix ``visual.``) on one GPU."""

    def __init__(self, sd: dict, device, prefix: str = "visual."):
        super().__init__()
        _lib.ensure_device(device)
        self.device = torch.device(device)
        g = lambda k: sd[prefix + k]  # noqa: E731
        conv = g("conv1.weight")
        self.width, self.patch = conv.shape[0], conv.shape[-1]
        pos = g("positional_embedding")
        self.grid = int(round((pos.shape[0] - 1) ** 0.5))
        self.image_size = self.grid * self.patch
        self.layers = _count_layers(sd, prefix + "transformer")
        self.out_dim = g("proj").shape[1]
        self.tokens = self.grid * self.grid + 1
        tensors = ([conv, g("class_embedding"), pos, g("ln_pre.weight"), g("ln_pre.bias")]
                   + _block_tensors(sd, prefix + "transformer", self.layers)
                   + [g("ln_post.weight"), g("ln_post.bias"), g("proj")])
        host = _host_f32(tensors)
        cfg = [self.width, self.layers, self.width // 64, self.patch, self.image_size,
               self.out_dim]
        h = _lib.ctypes.c_void_p()
        _lib.call("mpr_vit_create", _lib.int_array(cfg), len(cfg), _lib.tensor_array(host),
                  len(host), _lib.ctypes.byref(h))
        self._h = h

    def forward(self, img: torch.Tensor, mode: int = CLS, out: torch.Tensor = None,
                out_bstride: int = None) -> torch.Tensor:
        img = img.to(self.device, torch.float32, non_blocking=True).contiguous()
        B = img.shape[0]
        if tuple(img.shape[1:]) != (3, self.image_size, self.image_size):
            raise ValueError(f"expected images [B,3,{self.image_size},{self.image_size}], "
                             f"got {tuple(img.shape)}")
        if out is None:
            shape = (B, self.out_dim) if mode == CLS else (B, self.tokens, self.out_dim)
            out = torch.empty(shape, device=self.device, dtype=torch.float32)
            out_bstride = self.out_dim if mode == CLS else self.tokens * self.out_dim
        _lib.call("mpr_vit_forward", self._h, _lib.ptr(img), B, mode, _lib.ptr(out),
                  int(out_bstride), _lib.stream_ptr(self.device))
        return out

    __call__ = forward

    def _out(self, B, mode, out, out_bstride):
        if out is None:
            shape = (B, self.out_dim) if mode == CLS else (B, self.tokens, self.out_dim)
            out = torch.empty(shape, device=self.device, dtype=torch.float32)
            out_bstride = self.out_dim if mode == CLS else self.tokens * self.out_dim
        return out, out_bstride

    def forward_pair(self, other: "DeviceViT", img: torch.Tensor, mode: int = CLS,
                     other_mode: int = TOKENS, out: torch.Tensor = None, out_bstride: int = None,
                     other_out: torch.Tensor = None, other_bstride: int = None):
        """``self(img, mode)`` and ``other(img, other_mode)`` in one pass over the same images:
        im2col once, the two towers' projections of each layer as one grouped launch.  Results
        are identical to the two separate calls."""
        if other is self or other.device != self.device:
            raise ValueError("forward_pair needs a second ViT on the same device")
        img = img.to(self.device, torch.float32, non_blocking=True).contiguous()
        B = img.shape[0]
        if tuple(img.shape[1:]) != (3, self.image_size, self.image_size):
            raise ValueError(f"expected images [B,3,{self.image_size},{self.image_size}], "
                             f"got {tuple(img.shape)}")
        out, out_bstride = self._out(B, mode, out, out_bstride)
        other_out, other_bstride = other._out(B, other_mode, other_out, other_bstride)
        _lib.call("mpr_vit_forward_pair", self._h, mode, _lib.ptr(out), int(out_bstride),
                  other._h, other_mode, _lib.ptr(other_out), int(other_bstride), _lib.ptr(img),
                  B, _lib.stream_ptr(self.device))
        return out, other_out


def encode_towers(vit_a: "DeviceViT" = None, img: torch.Tensor = None, mode_a: int = CLS,
                  out_a=None, out_a_bstride=None, vit_b: "DeviceViT" = None,
                  mode_b: int = TOKENS, out_b=None, out_b_bstride=None,
                  text: "DeviceCLIPText" = None, tokens: torch.Tensor = None, out_t=None,
                  out_t_bstride=None, slot: int = 0):
    """One lockstep pass over a batch's CLIP towers (mpr_encode_towers): up to two ViTs over
    the same images and the text tower over clip.tokenize ids; each layer's projections share
    launches.  Bit-identical to the separate calls.  ``slot`` (0-3) picks the models'
    activation workspaces: passes on different slots may run concurrently on different streams.
    Returns (out_a, out_b, out_t)."""
    dev = (vit_a or text).device
    B = 0
    if vit_a is not None:
        img = img.to(dev, torch.float32, non_blocking=True).contiguous()
        B = img.shape[0]
        if tuple(img.shape[1:]) != (3, vit_a.image_size, vit_a.image_size):
            raise ValueError(f"expected images [B,3,{vit_a.image_size},{vit_a.image_size}], "
                             f"got {tuple(img.shape)}")
        out_a, out_a_bstride = vit_a._out(B, mode_a, out_a, out_a_bstride)
    if vit_b is not None:
        if vit_a is None or vit_b is vit_a or vit_b.device != dev:
            raise ValueError("vit_b needs a different vit_a on the same device")
        out_b, out_b_bstride = vit_b._out(B, mode_b, out_b, out_b_bstride)
    Bt, L, tok = 0, 0, None
    if text is not None:
        tok, L = text._tokens(tokens)
        Bt = tok.shape[0]
        if out_t is None:
            out_t = torch.empty((Bt, text.out_dim), device=dev, dtype=torch.float32)
            out_t_bstride = text.out_dim
    _lib.call("mpr_encode_towers",
              vit_a._h if vit_a is not None else None, mode_a, _lib.ptr(out_a),
              int(out_a_bstride or 0),
              vit_b._h if vit_b is not None else None, mode_b, _lib.ptr(out_b),
              int(out_b_bstride or 0),
              _lib.ptr(img if vit_a is not None else None), B,
              text._h if text is not None else None, _lib.ptr(tok), Bt, L, _lib.ptr(out_t),
              int(out_t_bstride or 0), int(slot), _lib.stream_ptr(dev))
    return out_a, out_b, out_t


def encode_towers_multi(vit_a: "DeviceViT", img: torch.Tensor, mode_a: int = CLS, out_a=None,
                        out_a_bstride=None, vit_b: "DeviceViT" = None, mode_b: int = TOKENS,
                        out_b=None, out_b_bstride=None, text: "DeviceCLIPText" = None,
                        tokens: list = (), out_t: list = None, out_t_bstride: list = None,
                        slot: int = 0):
    """encode_towers over several EQUAL-SIZED batches at once (mpr_encode_towers_multi): ``img``
    holds the batches' images concatenated (the ViTs run over all of them, choosing GEMM tiles
    for one batch's rows), ``tokens`` is a list of up to 2 per-batch clip.tokenize tensors (each
    its own text run, own length).  Every output row is bit-identical to the per-batch
    encode_towers call.  Returns (out_a, out_b, [out_t, ...])."""
    if len(tokens) > 2:
        raise ValueError(f"encode_towers_multi: {len(tokens)} text runs (at most 2)")
    if len(tokens) > 1 and any(t.shape[0] * len(tokens) != img.shape[0] for t in tokens):
        raise ValueError("encode_towers_multi: the batches must be of equal size "
                         f"({img.shape[0]} images, text runs of {[t.shape[0] for t in tokens]})")
    dev = vit_a.device
    img = img.to(dev, torch.float32, non_blocking=True).contiguous()
    B = img.shape[0]
    if tuple(img.shape[1:]) != (3, vit_a.image_size, vit_a.image_size):
        raise ValueError(f"expected images [B,3,{vit_a.image_size},{vit_a.image_size}], "
                         f"got {tuple(img.shape)}")
    out_a, out_a_bstride = vit_a._out(B, mode_a, out_a, out_a_bstride)
    if vit_b is not None:
        if vit_b is vit_a or vit_b.device != dev:
            raise ValueError("vit_b needs a different vit_a on the same device")
        out_b, out_b_bstride = vit_b._out(B, mode_b, out_b, out_b_bstride)
    toks, lens, outs, bss = [], [], [], []
    for j, t in enumerate(tokens):
        tok, L = text._tokens(t)
        toks.append(tok)
        lens.append(L)
        if out_t is None or out_t[j] is None:
            o = torch.empty((tok.shape[0], text.out_dim), device=dev, dtype=torch.float32)
            outs.append(o)
            bss.append(text.out_dim)
        else:
            outs.append(out_t[j])
            bss.append(int(out_t_bstride[j]))
    _lib.call("mpr_encode_towers_multi", vit_a._h, mode_a, _lib.ptr(out_a),
              int(out_a_bstride or 0), vit_b._h if vit_b is not None else None, mode_b,
              _lib.ptr(out_b), int(out_b_bstride or 0), _lib.ptr(img), B,
              text._h if text is not None else None, len(toks), _lib.tensor_array(toks),
              _lib.int_array([t.shape[0] for t in toks]), _lib.int_array(lens),
              _lib.tensor_array(outs), _lib.int_array(bss, _lib.ctypes.c_int64), int(slot),
              _lib.stream_ptr(dev))
    return out_a, out_b, outs


class DeviceCLIPText(_Handle):
    """CLIP text transformer (openai naming, no prefix) on one GPU."""

    def __init__(self, sd: dict, device, prefix: str = ""):
        super().__init__()
        _lib.ensure_device(device)
        self.device = torch.device(device)
        g = lambda k: sd[prefix + k]  # noqa: E731
        emb = g("token_embedding.weight")
        self.vocab, self.width = emb.shape
        self.context_length = g("positional_embedding").shape[0]
        self.layers = _count_layers(sd, prefix + "transformer")
        self.out_dim = g("text_projection").shape[1]
        tensors = ([emb, g("positional_embedding")]
                   + _block_tensors(sd, prefix + "transformer", self.layers)
                   + [g("ln_final.weight"), g("ln_final.bias"), g("text_projection")])
        host = _host_f32(tensors)
        cfg = [self.width, self.layers, self.width // 64, self.context_length, self.vocab,
               self.out_dim]
        h = _lib.ctypes.c_void_p()
        _lib.call("mpr_clip_text_create", _lib.int_array(cfg), len(cfg),
                  _lib.tensor_array(host), len(host), _lib.ctypes.byref(h))
        self._h = h

    def _tokens(self, tokens: torch.Tensor):
        """(device int32 ids, positions to run): only the leading positions up to the last EOT
        of the batch when the ids are on the host (causal attention makes the pooled output
        independent of later positions)."""
        if tokens.shape[1] != self.context_length:
            raise ValueError(f"expected tokens [B,{self.context_length}], got "
                             f"{tuple(tokens.shape)}")
        B = tokens.shape[0]
        if tokens.device.type == "cpu":
            seq_len = int(tokens.argmax(dim=1).max()) + 1 if B else 1
        else:
            seq_len = self.context_length
        return _lib.to_device_async(tokens, self.device, torch.int32).contiguous(), seq_len

    def forward(self, tokens: torch.Tensor, out: torch.Tensor = None,
                out_bstride: int = None) -> torch.Tensor:
        """tokens int [B, ctx] (host or device).  Runs only the leading positions up to the
        last EOT of the batch (causal attention makes the pooled output independent of the
        positions after each row's EOT)."""
        tok, seq_len = self._tokens(tokens)
        B = tok.shape[0]
        if out is None:
            out = torch.empty((B, self.out_dim), device=self.device, dtype=torch.float32)
            out_bstride = self.out_dim
        _lib.call("mpr_clip_text_forward", self._h, _lib.ptr(tok), B, seq_len, _lib.ptr(out),
                  int(out_bstride), _lib.stream_ptr(self.device))
        return out

    __call__ = forward
