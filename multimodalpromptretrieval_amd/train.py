"""Teacher-forced T5 training step on the device.

main.py:177-188 trains with ``loss = model(batch); loss.backward(); optimizer.step()``, and the
loss is ``T5_model(inputs_embeds=..., attention_mask=..., labels=...).loss``
(architectures/T5VisionModel.py:219-234): transformers' T5ForConditionalGeneration, whose
backward the reference leaves to torch autograd.  Here the whole T5 — encoder, decoder with
cross-attention, tied lm_head, token cross-entropy — is ONE autograd node (``T5LossFn``) whose
forward keeps the activations the backward needs and whose backward is written out layer by
layer on libmpr kernels (csrc/train.hip + the tiled fp32-accurate GEMM): every parameter
gradient and the gradient of ``inputs_embeds`` in a fixed summation order.  The question-token
embedding gather of prepare_input (:169) is a second node (``EmbedFn``) so its gradient reaches
``shared`` as in the reference (tied with the decoder input embedding and the lm_head).

Train mode (main.py:170 ``model.train()``): dropout at every site transformers' T5 applies it
(modeling_t5.py: T5Stack's dropout of the input embeddings and of the final-norm output,
T5Attention's dropout of the attention probabilities, T5LayerSelfAttention /
T5LayerCrossAttention / T5LayerFF's dropout of each sublayer's output before the residual add,
T5DenseActDense's dropout after the ReLU), rate ``dropout_rate`` (0.1 in the t5-small / t5-base
configs).  torch's RNG stream cannot be reproduced, so the masks are counter-based
(``mpr_dropout``: a hash of (seed, site, element index), one seed per forward) and the backward
regenerates them instead of storing them; parity is against the reference's forward/backward
with the same masks injected at transformers' sites (G12, tests/golden/make_goldens.py).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import _lib
from .t5 import relative_position_bucket

EPS = 1e-6
RELU = 2  # csrc ACT_RELU

# dropout sites: ((stack * 256 + layer) * 8 + kind), stack 0 = encoder / 1 = decoder, layer 255
# for the stack-level sites (input embeddings, final-norm output)
D_IN, D_FINAL, D_SELF_P, D_SELF_OUT, D_CROSS_P, D_CROSS_OUT, D_FFN_ACT, D_FFN_OUT = range(8)


def dropout_site(stack: int, layer: int, kind: int) -> int:
    return (stack * 256 + layer) * 8 + kind


class Dropout:
    """One forward's dropout: rate p, seed; ``args(site)`` = the mpr_dropout / attention
    (seed, site, thresh, scale) of a site (keep iff hash >= thresh = p * 2^24, kept * 1/(1-p))."""

    def __init__(self, p: float, seed: int):
        if not 0.0 < p < 1.0:
            raise ValueError(f"dropout rate {p}")
        self.p = float(p)
        self.seed = int(seed) & ((1 << 64) - 1)
        self.thresh = int(self.p * (1 << 24))
        self.scale = float(np.float32(1.0 / (1.0 - self.p)))

    def args(self, site: int):
        return (self.seed, int(site), self.thresh, self.scale)


NO_DROP = (0, 0, 0, 1.0)


def dropout(x, dr, site, residual=None):
    """residual + x * mask (a fresh tensor); dr None: x (+ residual)."""
    if dr is None:
        return x if residual is None else x + residual
    y = torch.empty_like(x)
    _lib.call("mpr_dropout", _lib.ptr(x), x.numel(), *dr.args(site), _lib.ptr(residual),
              _lib.ptr(y), _s())
    return y


def t5_param_names(n_enc: int, n_dec: int) -> list:
    """transformers names of the T5 parameters, in the order T5LossFn takes them (the tied
    embedding once, as shared.weight)."""
    names = ["shared.weight", "encoder.block.0.layer.0.SelfAttention.relative_attention_bias.weight",
             "decoder.block.0.layer.0.SelfAttention.relative_attention_bias.weight",
             "encoder.final_layer_norm.weight", "decoder.final_layer_norm.weight"]
    for i in range(n_enc):
        p = f"encoder.block.{i}.layer"
        names += [p + ".0.layer_norm.weight", p + ".0.SelfAttention.q.weight",
                  p + ".0.SelfAttention.k.weight", p + ".0.SelfAttention.v.weight",
                  p + ".0.SelfAttention.o.weight", p + ".1.layer_norm.weight",
                  p + ".1.DenseReluDense.wi.weight", p + ".1.DenseReluDense.wo.weight"]
    for i in range(n_dec):
        p = f"decoder.block.{i}.layer"
        names += [p + ".0.layer_norm.weight", p + ".0.SelfAttention.q.weight",
                  p + ".0.SelfAttention.k.weight", p + ".0.SelfAttention.v.weight",
                  p + ".0.SelfAttention.o.weight", p + ".1.layer_norm.weight",
                  p + ".1.EncDecAttention.q.weight", p + ".1.EncDecAttention.k.weight",
                  p + ".1.EncDecAttention.v.weight", p + ".1.EncDecAttention.o.weight",
                  p + ".2.layer_norm.weight", p + ".2.DenseReluDense.wi.weight",
                  p + ".2.DenseReluDense.wo.weight"]
    return names


def _layers(names_or_sd, stack: str) -> int:
    n = 0
    while f"{stack}.block.{n}.layer.0.layer_norm.weight" in names_or_sd:
        n += 1
    return n


# ---- thin wrappers over the ABI (current stream; fresh outputs) ---------------------------------
def _s():
    return _lib.stream_ptr()


def _empty(*shape, like):
    return torch.empty(shape, device=like.device, dtype=torch.float32)


def _cdiv(a: int, b: int) -> int:
    return -(-a // b)


def _splits(M: int, N: int, K: int) -> int:
    """K chunks for a GEMM with few output tiles over a long K (1: none): the dW GEMMs of a
    [512, 512] weight over ~2K rows fill 64 of 256 CUs, the tied lm_head's input gradient
    (M = B*T, N = d, K = vocab) 16."""
    tiles = _cdiv(M, 64) * _cdiv(N, 64)
    if tiles >= 128 or K < 1024:
        return 1
    return max(1, min(16, _cdiv(256, tiles), K // 256))


def gemm(A, W, R=None, act=0, ldw=None):
    """A [M, K] (row stride A.stride(0)) @ W[N, K]^T (+ R), fp32-accurate tiled GEMM (split
    over K into chunks summed in order when the output has few tiles, ``_splits``)."""
    M, K = A.shape
    N = W.shape[0]
    C = _empty(M, N, like=A)
    sp = _splits(M, N, K)
    if sp > 1:
        part = _empty(sp, M, N, like=A)
        _lib.call("mpr_gemm_f32_splitk", _lib.ptr(A), A.stride(0), _lib.ptr(W), W.stride(0),
                  _lib.ptr(C), N, M, N, K, _lib.ptr(R), N if R is not None else 0, act, sp,
                  _lib.ptr(part), _s())
        return C
    _lib.call("mpr_gemm_f32", _lib.ptr(A), A.stride(0), _lib.ptr(W), W.stride(0), _lib.ptr(C), N,
              M, N, K, _lib.ptr(R), N if R is not None else 0, act, _s())
    return C


def _r4(n: int) -> int:
    return (n + 3) // 4 * 4


def transpose(x, cols=None):
    """x [r, c] (row stride x.stride(0); only the first ``cols`` columns) -> [c, r4] (r4 = r
    rounded up to 4, zero columns: the GEMM K-alignment)."""
    r = x.shape[0]
    c = x.shape[1] if cols is None else cols
    out = _empty(c, _r4(r), like=x)
    _lib.call("mpr_transpose", _lib.ptr(x), r, c, x.stride(0), _lib.ptr(out), _r4(r), _s())
    return out


def linear_bwd(x, W, Wt, dy, dx_acc=None, need_dw=True, need_dx=True, xt=None):
    """y = x W^T: (dx (+ dx_acc), dW).  Wt = transpose(W) [K, N4], staged once per backward;
    dy's row stride must be N4 (N4 = N for every projection but the vocabulary); xt: x already
    transposed (shared by the projections of one input)."""
    N, K = W.shape
    dW = gemm(transpose(dy, N), xt if xt is not None else transpose(x)) if need_dw else None
    dx = gemm(dy, Wt, R=dx_acc) if need_dx else None
    return dx, dW


def rms_fwd(x, w, scale=1.0):
    M, D = x.shape
    y, r = _empty(M, D, like=x), _empty(M, like=x)
    _lib.call("mpr_rmsnorm_fwd", _lib.ptr(x), M, D, _lib.ptr(w), EPS, float(scale), _lib.ptr(y),
              _lib.ptr(r), _s())
    return y, r


def rms_bwd(x, w, rstd, dy, dx_acc=None, scale=1.0):
    """(dx (+ dx_acc, in place), dw)"""
    M, D = x.shape
    dx = dx_acc if dx_acc is not None else _empty(M, D, like=x)
    dw = _empty(D, like=x)
    part = _empty(_cdiv(M, 64), D, like=x)
    _lib.call("mpr_rmsnorm_bwd", _lib.ptr(x), M, D, _lib.ptr(w), _lib.ptr(rstd), _lib.ptr(dy),
              float(scale), _lib.ptr(dx), 1 if dx_acc is not None else 0, _lib.ptr(dw),
              _lib.ptr(part), _s())
    return dx, dw


def _qkv(t, j, inner):
    """The j-th inner-wide column block of a packed projection output t [rows, n * inner]."""
    return t[:, j * inner:(j + 1) * inner]


def attn_fwd(q, k, v, B, H, Lq, Lk, causal, mask, rel, R, drop=NO_DROP):
    """(dropout(P) V, P): P [B, H, Lq, Lk] kept before dropout (drop = Dropout.args(site)).
    q / k / v: [B*L, inner] column blocks of any row stride."""
    inner = q.shape[1]
    o = _empty(B * Lq, inner, like=q)
    P = _empty(B, H, Lq, Lk, like=q)
    qs, ks, vs = q.stride(0), k.stride(0), v.stride(0)
    _lib.call("mpr_attn_train_fwd", _lib.ptr(q), Lq * qs, qs, _lib.ptr(k), Lk * ks, ks,
              _lib.ptr(v), Lk * vs, vs, B, H, Lq, Lk, int(causal), _lib.ptr(mask), _lib.ptr(rel),
              R, _lib.ptr(o), Lq * inner, inner, _lib.ptr(P), *drop, _s())
    return o, P


def attn_bwd(q, k, v, P, do, B, H, Lq, Lk, drel, R, drop=NO_DROP, dq=None, dk=None, dv=None):
    """(dq, dk, dv); given outputs (column blocks of packed buffers) are written in place."""
    inner = q.shape[1]
    dS = torch.empty_like(P)
    dq = dq if dq is not None else _empty(B * Lq, inner, like=q)
    dk = dk if dk is not None else _empty(B * Lk, inner, like=q)
    dv = dv if dv is not None else _empty(B * Lk, inner, like=q)
    qs, ks, vs = q.stride(0), k.stride(0), v.stride(0)
    dqs, dks, dvs = dq.stride(0), dk.stride(0), dv.stride(0)
    _lib.call("mpr_attn_train_bwd", _lib.ptr(q), Lq * qs, qs, _lib.ptr(k), Lk * ks, ks,
              _lib.ptr(v), Lk * vs, vs, B, H, Lq, Lk, _lib.ptr(P), _lib.ptr(do), Lq * inner,
              inner, _lib.ptr(dS), _lib.ptr(dq), Lq * dqs, dqs, _lib.ptr(dk), Lk * dks, dks,
              _lib.ptr(dv), Lk * dvs, dvs, _lib.ptr(drel), R, *drop, _s())
    return dq, dk, dv


def _grouped(ids: np.ndarray):
    """Positions of each distinct id (stable order): (uniq, offs, pos) int32 for mpr_embed_bwd."""
    ids = ids.reshape(-1).astype(np.int64)
    order = np.argsort(ids, kind="stable")
    uniq, counts = np.unique(ids[order], return_counts=True)
    offs = np.concatenate([[0], np.cumsum(counts)])
    return uniq.astype(np.int32), offs.astype(np.int32), order.astype(np.int32)


def _upload_i32(dev, *arrays):
    """Host int arrays -> int32 device tensors through ONE pinned, non-blocking copy."""
    flat = np.concatenate([np.asarray(a, dtype=np.int32).reshape(-1) for a in arrays])
    t = _lib.to_device_async(torch.from_numpy(flat), dev)
    out, o = [], 0
    for a in arrays:
        n = int(np.asarray(a).size)
        out.append(t[o:o + n])
        o += n
    return out


def embed_bwd_into(dW, ids_host: np.ndarray, dY):
    uniq, offs, pos = _grouped(ids_host)
    u, o, p = _upload_i32(dY.device, uniq, offs, pos)
    _lib.call("mpr_embed_bwd", _lib.ptr(dY), dY.shape[-1], _lib.ptr(u), _lib.ptr(o), _lib.ptr(p),
              len(uniq), _lib.ptr(dW), _s())


def gather_rows(table, ids_dev):
    n = ids_dev.numel()
    d = table.shape[1]
    out = _empty(n, d, like=table)
    _lib.call("mpr_gather_rows", _lib.ptr(table), _lib.ptr(ids_dev), n, d, _lib.ptr(out), _s())
    return out


def _host_ids(ids) -> np.ndarray:
    """Token ids as a host array (prepare_input's tokenizer output is a host tensor already; a
    device tensor costs a wait for the GPU here)."""
    return ids.detach().cpu().numpy() if ids.device.type != "cpu" else ids.detach().numpy()


class EmbedFn(torch.autograd.Function):
    """``T5_model.shared(input_ids)`` (architectures/T5VisionModel.py:169) with its gradient."""

    @staticmethod
    def forward(ctx, weight, ids):
        ids_dev = _lib.to_device_async(ids, weight.device, torch.int32).contiguous()
        ctx.ids_host = _host_ids(ids) if ids.device.type == "cpu" else ids.detach()
        ctx.wshape = weight.shape
        return gather_rows(weight.detach(), ids_dev.view(-1)).view(*ids.shape, weight.shape[1])

    @staticmethod
    def backward(ctx, dy):
        dW = torch.zeros(ctx.wshape, device=dy.device, dtype=torch.float32)
        ids = ctx.ids_host if isinstance(ctx.ids_host, np.ndarray) else _host_ids(ctx.ids_host)
        embed_bwd_into(dW, ids, dy.contiguous().view(-1, ctx.wshape[1]))
        return dW, None


def embed_rows(weight, ids):
    return EmbedFn.apply(weight, ids)


class T5LossFn(torch.autograd.Function):
    """T5ForConditionalGeneration(inputs_embeds, attention_mask, labels).loss and its backward.
    ``params`` in ``t5_param_names`` order."""

    @staticmethod
    def forward(ctx, cfg, inputs_embeds, mask, labels, *params):
        runner = _Runner(cfg, params)
        loss, tape = runner.forward(inputs_embeds.detach(), mask, labels)
        ctx.runner, ctx.tape = runner, tape
        return loss

    @staticmethod
    def backward(ctx, dloss):
        # dloss stays on the device (the cross-entropy kernel reads it): no host wait
        needs = ctx.needs_input_grad
        dl = dloss.detach().to(torch.float32).contiguous()
        d_emb, grads = ctx.runner.backward(ctx.tape, dl, needs[4:], needs[1])
        ctx.tape = None
        return (None, d_emb, None, None, *grads)


class T5Config:
    def __init__(self, names, shapes, num_heads, max_distance=128, scale_out=True):
        self.n_enc = _layers(names, "encoder")
        self.n_dec = _layers(names, "decoder")
        self.vocab, self.d = shapes["shared.weight"]
        self.num_buckets, self.H = shapes[
            "encoder.block.0.layer.0.SelfAttention.relative_attention_bias.weight"]
        assert self.H == num_heads
        self.inner = shapes["encoder.block.0.layer.0.SelfAttention.q.weight"][0]
        self.max_distance = max_distance
        self.scale_out = scale_out
        self.dropout = None  # Dropout in train mode
        self._luts = {}

    def lut(self, R, bidirectional, device):
        key = (R, bidirectional, str(device))
        if key not in self._luts:
            rel = torch.arange(-R, R + 1, dtype=torch.long)
            self._luts[key] = relative_position_bucket(rel, bidirectional, self.num_buckets,
                                                       self.max_distance).to(
                device, torch.int32).contiguous()
        return self._luts[key]


class _Runner:
    def __init__(self, cfg: T5Config, params):
        self.c = cfg
        self.names = t5_param_names(cfg.n_enc, cfg.n_dec)
        self.p = {n: t.detach().contiguous() for n, t in zip(self.names, params)}

    # ---- forward --------------------------------------------------------------------------------
    def cat_w(self, names):
        """The named [n, K] weights stacked row-wise: one GEMM computes their projections side by
        side (q | k | v of a layer; every decoder layer's cross k | v of the encoder output)."""
        return torch.cat([self.p[n] for n in names], 0)

    def forward(self, emb, mask, labels):
        c, p = self.c, self.p
        dr = c.dropout  # a Dropout in train mode, else None
        B, L, d = emb.shape
        H, inner = c.H, c.inner
        dev = emb.device
        lab_host = _host_ids(labels).astype(np.int64)
        T = lab_host.shape[1]
        dec_ids = np.zeros_like(lab_host)
        dec_ids[:, 1:] = lab_host[:, :-1]
        dec_ids[dec_ids == -100] = 0  # shift_right (decoder_start_token_id 0, pad 0)
        ids_dev, lab32 = _upload_i32(dev, dec_ids, lab_host)
        n_valid = int((lab_host != -100).sum())
        Re, Rd = max(L, 1), max(T, 1)
        lut_e, lut_d = c.lut(Re, True, dev), c.lut(Rd, False, dev)
        rel_e = _empty(2 * Re + 1, H, like=emb)
        _lib.call("mpr_rel_gather", _lib.ptr(p[self.names[1]]), _lib.ptr(lut_e), Re, H,
                  _lib.ptr(rel_e), _s())
        rel_d = _empty(2 * Rd + 1, H, like=emb)
        _lib.call("mpr_rel_gather", _lib.ptr(p[self.names[2]]), _lib.ptr(lut_d), Rd, H,
                  _lib.ptr(rel_d), _s())
        maskf = _lib.to_device_async(mask, dev, torch.float32).contiguous()
        tape = {"B": B, "L": L, "T": T, "Re": Re, "Rd": Rd, "lut_e": lut_e, "lut_d": lut_d,
                "mask": maskf, "dec_ids": dec_ids, "enc": [], "dec": []}

        def pdrop(stack, layer, kind):  # attention-probability dropout arguments
            return dr.args(dropout_site(stack, layer, kind)) if dr else NO_DROP

        def proj_res(a, W, R, site):  # R + dropout(a W^T)  (the sublayer output's dropout)
            if dr is None:
                return gemm(a, W, R=R)
            return dropout(gemm(a, W), dr, site, residual=R)

        # encoder
        x = dropout(emb.contiguous().view(B * L, d), dr, dropout_site(0, 255, D_IN))
        for i in range(c.n_enc):
            pre = f"encoder.block.{i}.layer"
            t = {"x0": x}
            t["n1"], t["r1"] = rms_fwd(x, p[pre + ".0.layer_norm.weight"])
            t["Wqkv"] = self.cat_w([pre + f".0.SelfAttention.{z}.weight" for z in "qkv"])
            t["qkv"] = gemm(t["n1"], t["Wqkv"])
            q, k, v = (_qkv(t["qkv"], j, inner) for j in range(3))
            t["a"], t["P"] = attn_fwd(q, k, v, B, H, L, L, False, maskf, rel_e, Re,
                                      pdrop(0, i, D_SELF_P))
            t["x1"] = proj_res(t["a"], p[pre + ".0.SelfAttention.o.weight"], x,
                               dropout_site(0, i, D_SELF_OUT))
            t["n2"], t["r2"] = rms_fwd(t["x1"], p[pre + ".1.layer_norm.weight"])
            t["f"] = gemm(t["n2"], p[pre + ".1.DenseReluDense.wi.weight"], act=RELU)
            fd = dropout(t["f"], dr, dropout_site(0, i, D_FFN_ACT))
            x = proj_res(fd, p[pre + ".1.DenseReluDense.wo.weight"], t["x1"],
                         dropout_site(0, i, D_FFN_OUT))
            tape["enc"].append(t)
        tape["enc_in"] = x
        enc, tape["enc_r"] = rms_fwd(x, p["encoder.final_layer_norm.weight"])
        enc = dropout(enc, dr, dropout_site(0, 255, D_FINAL))
        tape["enc_out"] = enc
        # every decoder layer's cross-attention k | v of the encoder output in one GEMM
        ckv_names = [f"decoder.block.{i}.layer.1.EncDecAttention.{z}.weight"
                     for i in range(c.n_dec) for z in "kv"]
        tape["Wckv"] = self.cat_w(ckv_names) if c.n_dec else None
        tape["ckv"] = gemm(enc, tape["Wckv"]) if c.n_dec else None
        # decoder
        g = dropout(gather_rows(p["shared.weight"], ids_dev), dr, dropout_site(1, 255, D_IN))
        for i in range(c.n_dec):
            pre = f"decoder.block.{i}.layer"
            t = {"g0": g}
            t["n1"], t["r1"] = rms_fwd(g, p[pre + ".0.layer_norm.weight"])
            t["Wqkv"] = self.cat_w([pre + f".0.SelfAttention.{z}.weight" for z in "qkv"])
            t["qkv"] = gemm(t["n1"], t["Wqkv"])
            q, k, v = (_qkv(t["qkv"], j, inner) for j in range(3))
            t["a"], t["P"] = attn_fwd(q, k, v, B, H, T, T, True, None, rel_d, Rd,
                                      pdrop(1, i, D_SELF_P))
            t["g1"] = proj_res(t["a"], p[pre + ".0.SelfAttention.o.weight"], g,
                               dropout_site(1, i, D_SELF_OUT))
            t["n2"], t["r2"] = rms_fwd(t["g1"], p[pre + ".1.layer_norm.weight"])
            t["cq"] = gemm(t["n2"], p[pre + ".1.EncDecAttention.q.weight"])
            ck, cv = _qkv(tape["ckv"], 2 * i, inner), _qkv(tape["ckv"], 2 * i + 1, inner)
            t["ca"], t["cP"] = attn_fwd(t["cq"], ck, cv, B, H, T, L, False, maskf, None, 0,
                                        pdrop(1, i, D_CROSS_P))
            t["g2"] = proj_res(t["ca"], p[pre + ".1.EncDecAttention.o.weight"], t["g1"],
                               dropout_site(1, i, D_CROSS_OUT))
            t["n3"], t["r3"] = rms_fwd(t["g2"], p[pre + ".2.layer_norm.weight"])
            t["f"] = gemm(t["n3"], p[pre + ".2.DenseReluDense.wi.weight"], act=RELU)
            fd = dropout(t["f"], dr, dropout_site(1, i, D_FFN_ACT))
            g = proj_res(fd, p[pre + ".2.DenseReluDense.wo.weight"], t["g2"],
                         dropout_site(1, i, D_FFN_OUT))
            tape["dec"].append(t)
        tape["dec_in"] = g
        s = c.d ** -0.5 if c.scale_out else 1.0
        tape["s"] = s
        hs, tape["dec_r"] = rms_fwd(g, p["decoder.final_layer_norm.weight"], scale=s)
        hs = dropout(hs, dr, dropout_site(1, 255, D_FINAL))
        tape["hs"] = hs
        logits = gemm(hs, p["shared.weight"])
        tape["logits"] = logits
        tape["lab"], tape["n_valid"] = lab32, n_valid
        row_loss = _empty(B * T, like=emb)
        loss = torch.empty((), device=dev, dtype=torch.float32)
        _lib.call("mpr_ce_train", _lib.ptr(logits), B * T, c.vocab, _lib.ptr(lab32),
                  1.0 / max(n_valid, 1) if n_valid else float("nan"), 0.0, None,
                  _lib.ptr(row_loss), _lib.ptr(loss), None, 0, _s())
        return loss, tape

    # ---- backward -------------------------------------------------------------------------------
    def backward(self, tape, dloss, need_params, need_emb):
        """dloss: the loss gradient as a device scalar."""
        c, p = self.c, self.p
        dr = c.dropout
        B, L, T, H, inner = tape["B"], tape["L"], tape["T"], c.H, c.inner
        nm = self.names
        idx = {n: i for i, n in enumerate(nm)}
        grads = [None] * len(nm)

        def want(name):
            return bool(need_params[idx[name]])

        def put(name, g):
            if want(name):
                grads[idx[name]] = g

        def put_rows(names, dW):  # the row blocks of a stacked weight's gradient
            n = dW.shape[0] // len(names)
            for j, name in enumerate(names):
                put(name, dW[j * n:(j + 1) * n])

        def pdrop(stack, layer, kind):
            return dr.args(dropout_site(stack, layer, kind)) if dr else NO_DROP

        def dmask(g, stack, layer, kind):  # gradient through a dropout site: g * mask
            return dropout(g, dr, dropout_site(stack, layer, kind))

        dev = tape["logits"].device
        wt = {}

        def Wt(name):  # W^T once per backward
            if name not in wt:
                wt[name] = transpose(p[name])
            return wt[name]

        def self_attn_bwd(t, da, stack, i, Lx, causal_R, drel, names, x_name):
            """The self-attention block's projections from da: dn (input of q|k|v) and the
            stacked q|k|v weight gradient (one GEMM each over the packed dq|dk|dv)."""
            q, k, v = (_qkv(t["qkv"], j, inner) for j in range(3))
            dqkv = _empty(B * Lx, 3 * inner, like=da)
            attn_bwd(q, k, v, t["P"], da, B, H, Lx, Lx, drel, causal_R, pdrop(stack, i, D_SELF_P),
                     *(_qkv(dqkv, j, inner) for j in range(3)))
            dn = gemm(dqkv, transpose(t["Wqkv"]))
            if any(want(n) for n in names):
                put_rows(names, gemm(transpose(dqkv), transpose(t[x_name])))
            return dn

        # loss -> logits
        logits = tape["logits"]
        V4 = _r4(c.vocab)  # dlogits rows padded with zeros: the lm_head dx GEMM's K
        dlogits = _empty(B * T, V4, like=logits)
        row_loss = _empty(B * T, like=logits)
        scratch = torch.empty((), device=dev, dtype=torch.float32)
        nv = max(tape["n_valid"], 1)
        _lib.call("mpr_ce_train", _lib.ptr(logits), B * T, c.vocab, _lib.ptr(tape["lab"]),
                  1.0 / nv, 1.0 / nv, _lib.ptr(dloss), _lib.ptr(row_loss), _lib.ptr(scratch),
                  _lib.ptr(dlogits), V4, _s())
        tape["logits"] = None
        # lm_head (tied): logits = hs shared^T; its weight gradient opens the tied gradient
        dhs, d_shared = linear_bwd(tape["hs"], p["shared.weight"], Wt("shared.weight"), dlogits)
        del dlogits
        dg, dw = rms_bwd(tape["dec_in"], p["decoder.final_layer_norm.weight"], tape["dec_r"],
                         dmask(dhs, 1, 255, D_FINAL), scale=tape["s"])
        put("decoder.final_layer_norm.weight", dw)
        drel_d = torch.zeros((2 * tape["Rd"] + 1, H), device=dev, dtype=torch.float32)
        # every layer's cross k | v gradient lands in one packed buffer: one GEMM each for the
        # encoder output's gradient and the stacked weight gradient after the loop
        dckv = _empty(B * L, 2 * c.n_dec * inner, like=tape["enc_out"]) if c.n_dec else None
        for i in reversed(range(c.n_dec)):
            pre = f"decoder.block.{i}.layer"
            t = tape["dec"][i]
            # FFN: g = g2 + drop(drop(relu(n3 Wi^T)) Wo^T)
            wo, wi = pre + ".2.DenseReluDense.wo.weight", pre + ".2.DenseReluDense.wi.weight"
            fd = dropout(t["f"], dr, dropout_site(1, i, D_FFN_ACT))
            df, dW = linear_bwd(fd, p[wo], Wt(wo), dmask(dg, 1, i, D_FFN_OUT), need_dw=want(wo))
            put(wo, dW)
            del fd
            df = dmask(df, 1, i, D_FFN_ACT)
            _lib.call("mpr_relu_bwd", _lib.ptr(t["f"]), _lib.ptr(df), df.numel(), _lib.ptr(df),
                      _s())
            dn3, dW = linear_bwd(t["n3"], p[wi], Wt(wi), df, need_dw=want(wi))
            put(wi, dW)
            ln = pre + ".2.layer_norm.weight"
            dg2, dw = rms_bwd(t["g2"], p[ln], t["r3"], dn3, dx_acc=dg)
            put(ln, dw)
            # cross-attention: g2 = g1 + drop(attn(n2 Wq^T, enc Wk^T, enc Wv^T) Wo^T)
            co = pre + ".1.EncDecAttention.o.weight"
            dca, dW = linear_bwd(t["ca"], p[co], Wt(co), dmask(dg2, 1, i, D_CROSS_OUT),
                                 need_dw=want(co))
            put(co, dW)
            ck, cv = _qkv(tape["ckv"], 2 * i, inner), _qkv(tape["ckv"], 2 * i + 1, inner)
            dcq, _, _ = attn_bwd(t["cq"], ck, cv, t["cP"], dca, B, H, T, L, None, 0,
                                 pdrop(1, i, D_CROSS_P), dk=_qkv(dckv, 2 * i, inner),
                                 dv=_qkv(dckv, 2 * i + 1, inner))
            cq = pre + ".1.EncDecAttention.q.weight"
            dn2, dW = linear_bwd(t["n2"], p[cq], Wt(cq), dcq, need_dw=want(cq))
            put(cq, dW)
            ln = pre + ".1.layer_norm.weight"
            dg1, dw = rms_bwd(t["g1"], p[ln], t["r2"], dn2, dx_acc=dg2)
            put(ln, dw)
            # self-attention: g1 = g0 + drop(attn(n1 Wq^T, n1 Wk^T, n1 Wv^T; causal, bias) Wo^T)
            so = pre + ".0.SelfAttention.o.weight"
            da, dW = linear_bwd(t["a"], p[so], Wt(so), dmask(dg1, 1, i, D_SELF_OUT),
                                need_dw=want(so))
            put(so, dW)
            dn1 = self_attn_bwd(t, da, 1, i, T, tape["Rd"], drel_d,
                                [pre + f".0.SelfAttention.{z}.weight" for z in "qkv"], "n1")
            ln = pre + ".0.layer_norm.weight"
            dg, dw = rms_bwd(t["g0"], p[ln], t["r1"], dn1, dx_acc=dg1)
            put(ln, dw)
            tape["dec"][i] = None
        # decoder input embedding (tied), through its dropout
        embed_bwd_into(d_shared, tape["dec_ids"], dmask(dg, 1, 255, D_IN))
        put("shared.weight", d_shared)
        dtab = torch.zeros_like(p[nm[2]])
        _lib.call("mpr_rel_scatter", _lib.ptr(drel_d), _lib.ptr(tape["lut_d"]), tape["Rd"],
                  c.num_buckets, H, _lib.ptr(dtab), _s())
        put(nm[2], dtab)
        # the cross k | v projections of every layer: the encoder output's gradient and the
        # stacked weight gradient
        d_enc = None
        if c.n_dec:
            d_enc = gemm(dckv, transpose(tape["Wckv"]))
            ckv_names = [f"decoder.block.{i}.layer.1.EncDecAttention.{z}.weight"
                         for i in range(c.n_dec) for z in "kv"]
            if any(want(n) for n in ckv_names):
                put_rows(ckv_names, gemm(transpose(dckv), transpose(tape["enc_out"])))
            del dckv
        # encoder
        dx, dw = rms_bwd(tape["enc_in"], p["encoder.final_layer_norm.weight"], tape["enc_r"],
                         dmask(d_enc, 0, 255, D_FINAL))
        put("encoder.final_layer_norm.weight", dw)
        drel_e = torch.zeros((2 * tape["Re"] + 1, H), device=dev, dtype=torch.float32)
        for i in reversed(range(c.n_enc)):
            pre = f"encoder.block.{i}.layer"
            t = tape["enc"][i]
            wo, wi = pre + ".1.DenseReluDense.wo.weight", pre + ".1.DenseReluDense.wi.weight"
            fd = dropout(t["f"], dr, dropout_site(0, i, D_FFN_ACT))
            df, dW = linear_bwd(fd, p[wo], Wt(wo), dmask(dx, 0, i, D_FFN_OUT), need_dw=want(wo))
            put(wo, dW)
            del fd
            df = dmask(df, 0, i, D_FFN_ACT)
            _lib.call("mpr_relu_bwd", _lib.ptr(t["f"]), _lib.ptr(df), df.numel(), _lib.ptr(df),
                      _s())
            dn2, dW = linear_bwd(t["n2"], p[wi], Wt(wi), df, need_dw=want(wi))
            put(wi, dW)
            ln = pre + ".1.layer_norm.weight"
            dx1, dw = rms_bwd(t["x1"], p[ln], t["r2"], dn2, dx_acc=dx)
            put(ln, dw)
            so = pre + ".0.SelfAttention.o.weight"
            da, dW = linear_bwd(t["a"], p[so], Wt(so), dmask(dx1, 0, i, D_SELF_OUT),
                                need_dw=want(so))
            put(so, dW)
            dn1 = self_attn_bwd(t, da, 0, i, L, tape["Re"], drel_e,
                                [pre + f".0.SelfAttention.{z}.weight" for z in "qkv"], "n1")
            ln = pre + ".0.layer_norm.weight"
            dx, dw = rms_bwd(t["x0"], p[ln], t["r1"], dn1, dx_acc=dx1)
            put(ln, dw)
            tape["enc"][i] = None
        dtab = torch.zeros_like(p[nm[1]])
        _lib.call("mpr_rel_scatter", _lib.ptr(drel_e), _lib.ptr(tape["lut_e"]), tape["Re"],
                  c.num_buckets, H, _lib.ptr(dtab), _s())
        put(nm[1], dtab)
        d_emb = dmask(dx, 0, 255, D_IN).view(B, L, c.d) if need_emb else None
        return d_emb, grads


def t5_loss(named_params: dict, inputs_embeds, attention_mask, labels, num_heads: int,
            scale_out: bool = True, dropout_rate: float = 0.0, dropout_seed: int = None):
    """Differentiable T5ForConditionalGeneration(...).loss over ``named_params`` (transformers
    names -> Parameters; the tied embedding as shared.weight).  ``dropout_rate`` > 0: train
    mode's dropout at transformers' sites, masks from ``dropout_seed`` (default: drawn from
    torch's global generator, so torch.manual_seed fixes them)."""
    names = list(named_params)
    n_enc, n_dec = _layers(names, "encoder"), _layers(names, "decoder")
    order = t5_param_names(n_enc, n_dec)
    shapes = {n: tuple(named_params[n].shape) for n in order}
    cfg = T5Config(order, shapes, num_heads, scale_out=scale_out)
    if dropout_rate > 0.0:
        if dropout_seed is None:
            dropout_seed = int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64))
        cfg.dropout = Dropout(dropout_rate, dropout_seed)
    return T5LossFn.apply(cfg, inputs_embeds, attention_mask, labels,
                          *[named_params[n] for n in order])
