"""Teacher-forced T5 training step on the device.

main.py:177-188 trains with ``loss = model(batch); loss.backward(); optimizer.step()``, and the
loss is ``T5_model(inputs_embeds=..., attention_mask=..., labels=...).loss``
(architectures/T5VisionModel.py:219-234): transformers' T5ForConditionalGeneration, whose
backward the reference leaves to torch autograd.  Here the whole T5 — encoder, decoder with
cross-attention, tied lm_head, token cross-entropy — is ONE autograd node (``T5LossFn``) whose
forward and backward are each ONE call into libmpr's native trainer (csrc/trainer.hip: the
activations on a device tape, the backward written out layer by layer on the train.hip kernels and
the tiled fp32-accurate GEMM, every parameter gradient and the gradient of ``inputs_embeds`` in a
fixed summation order, written into one flat gradient buffer).  The question-token embedding
gather of prepare_input (:169) is a second node (``EmbedFn``) so its gradient reaches ``shared``
as in the reference (tied with the decoder input embedding and the lm_head).

Train mode (main.py:170 ``model.train()``): dropout at every site transformers' T5 applies it
(modeling_t5.py: T5Stack's dropout of the input embeddings and of the final-norm output,
T5Attention's dropout of the attention probabilities, T5LayerSelfAttention /
T5LayerCrossAttention / T5LayerFF's dropout of each sublayer's output before the residual add,
T5DenseActDense's dropout after the ReLU), rate ``dropout_rate`` (0.1 in the t5-small / t5-base
configs).  torch's RNG stream cannot be reproduced, so the masks are counter-based
(``mpr_dropout``: a hash of (seed, site, element index), one seed per forward) and the backward
regenerates them instead of storing them; parity is against the reference's forward/backward
with the same masks injected at transformers' sites (G12, tests/golden/make_goldens.py).

No host wait inside a step: the labels and decoder ids stay on the host (they come from the
tokenizer there) and go up through one pinned non-blocking copy; the loss gradient is read on the
device.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import _lib
from .t5 import relative_position_bucket

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


class _Tape:
    """A forward's activations on the native trainer: released when the backward has run or the
    autograd graph is dropped without one."""

    def __init__(self, trainer, tid: int):
        self.trainer, self.tid = trainer, tid
        self.done = None  # a speculative backward's completion event (T5LossFn.forward)

    def release(self):
        if self.tid is not None and _lib._lib is not None:
            if self.done is not None:  # the arena's next user comes after that backward
                torch.cuda.current_stream().wait_event(self.done)
            _lib.call("mpr_t5_train_release", self.trainer, self.tid)
        self.tid = None

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass


class T5LossFn(torch.autograd.Function):
    """T5ForConditionalGeneration(inputs_embeds, attention_mask, labels).loss and its backward.
    ``params`` in ``t5_param_names`` order."""

    @staticmethod
    def forward(ctx, cfg, inputs_embeds, mask, labels, *params):
        dev = inputs_embeds.device
        B, L, d = inputs_embeds.shape
        lab_host = _host_ids(labels).astype(np.int64)
        T = lab_host.shape[1]
        dec_ids = np.zeros_like(lab_host)
        dec_ids[:, 1:] = lab_host[:, :-1]
        dec_ids[dec_ids == -100] = 0  # shift_right (decoder_start_token_id 0, pad 0)
        ids_dev, lab32 = _upload_i32(dev, dec_ids, lab_host)
        n_valid = int((lab_host != -100).sum())
        emb = inputs_embeds.detach().to(torch.float32).contiguous()
        maskf = _lib.to_device_async(mask, dev, torch.float32).contiguous()
        ps = [p.detach().to(torch.float32).contiguous() for p in params]
        parr = _lib.tensor_array(ps)
        loss = torch.empty((), device=dev, dtype=torch.float32)
        dr = cfg.dropout
        seed, thresh, scale = (dr.seed, dr.thresh, dr.scale) if dr is not None else (0, 0, 1.0)
        tr = cfg.trainer(dev)
        _after_spec(tr, dev)
        tid = _lib.ctypes.c_int32()
        _lib.call("mpr_t5_train_forward", tr, parr, len(ps), _lib.ptr(emb), _lib.ptr(maskf), B, L,
                  _lib.ptr(ids_dev), _lib.ptr(lab32), T,
                  1.0 / max(n_valid, 1) if n_valid else float("nan"), seed, thresh, scale,
                  _lib.ptr(loss), _lib.ctypes.byref(tid), _s())
        ctx.tape = _Tape(tr, tid.value)
        # the tape points into these: alive until the backward
        ctx.keep = (emb, maskf, ids_dev, lab32, ps, parr)
        ctx.dec_ids, ctx.n_valid, ctx.shape = dec_ids, n_valid, (B, L, d)
        ctx.spec = None
        # needs_input_grad reflects requires_grad, not grad mode: a forward under no_grad (a
        # train-mode forward whose loss is only read) is never backwarded, so it enqueues none
        if (speculative_backward() and cfg.grad_enabled and any(ctx.needs_input_grad) and
                dev.type == "cuda"):
            # main.py:177-186 runs model(batch), then predict(batch), then loss.backward(): the
            # backward for a loss gradient of 1 is enqueued now on a side stream ordered after
            # this forward, so it runs on the GPU beside predict()'s decode (which the host
            # waits for) instead of after it; backward() then scales these gradients by the
            # real loss gradient (x 1.0 when it is loss.backward(): the same bits).
            cur = torch.cuda.current_stream(dev)
            side = _spec_stream(dev)
            side.wait_stream(cur)
            # the tape's inputs were allocated on `cur`: if the graph is dropped without a
            # backward they are freed while the side stream may still read them
            for t in (emb, maskf, ids_dev, lab32, *ps):
                t.record_stream(side)
            with torch.cuda.stream(side):
                out = T5LossFn._native_backward(ctx, torch.ones((), device=dev))
                done = torch.cuda.Event()
                done.record(side)
            ctx.spec = (out, done)
            ctx.tape.done = done
            _LAST_SPEC[tr.value] = done
        return loss

    @staticmethod
    def backward(ctx, dloss):
        # dloss stays on the device (the cross-entropy kernel reads it): no host wait
        dl = dloss.detach().to(torch.float32).contiguous()
        if ctx.spec is not None:
            (d_emb, grads, flat), done = ctx.spec
            cur = torch.cuda.current_stream(dl.device)
            cur.wait_event(done)
            for t in (flat, d_emb):
                if t is not None:
                    t.record_stream(cur)
                    t.mul_(dl)
            ctx.spec = None
        else:
            d_emb, grads, _ = T5LossFn._native_backward(ctx, dl)
        ctx.tape.release()
        ctx.keep = None
        return (None, d_emb, None, None, *grads)

    @staticmethod
    def _native_backward(ctx, dl):
        """mpr_t5_train_backward of the tape for loss gradient ``dl`` (device scalar) on the
        current stream: (d_emb or None, per-parameter gradients, their flat buffer)."""
        needs = ctx.needs_input_grad
        emb, maskf, ids_dev, lab32, ps, parr = ctx.keep
        dev = emb.device
        # every gradient in one flat buffer (views): a stacked weight's gradient (q | k | v of a
        # layer) lands with one GEMM when its parts are adjacent
        sizes = [p.numel() for p in ps]
        flat = torch.empty(sum(sizes), device=dev, dtype=torch.float32)
        grads, gptr, off = [], (_lib.ctypes.c_void_p * len(ps))(), 0
        for i, (p, n) in enumerate(zip(ps, sizes)):
            if needs[4 + i]:
                g = flat[off:off + n].view(p.shape)
                grads.append(g)
                gptr[i] = g.data_ptr()
            else:
                grads.append(None)
                gptr[i] = None
            off += n
        uniq, offs, pos = _grouped(ctx.dec_ids)
        u, o, q = _upload_i32(dev, uniq, offs, pos)
        d_emb = torch.empty(ctx.shape, device=dev, dtype=torch.float32) if needs[1] else None
        tr = ctx.tape.trainer
        _lib.call("mpr_t5_train_backward", tr, ctx.tape.tid, parr, len(ps), _lib.ptr(dl),
                  1.0 / max(ctx.n_valid, 1), _lib.ptr(u), _lib.ptr(o), _lib.ptr(q), len(uniq),
                  gptr, _lib.ptr(d_emb), _s())
        return d_emb, grads, flat


def speculative_backward() -> bool:
    """T5LossFn's backward enqueued with its forward (MPR_SPEC_BACKWARD=0: at backward())."""
    return os.environ.get("MPR_SPEC_BACKWARD", "1") != "0"


_SPEC_STREAMS = {}
_LAST_SPEC = {}  # trainer -> its latest speculative backward's completion event


def _after_spec(tr, dev):
    """Order the current stream after the trainer's latest speculative backward: the trainer's
    scratch is shared by its calls, which must not overlap."""
    ev = _LAST_SPEC.get(tr.value)
    if ev is not None and dev.type == "cuda":
        torch.cuda.current_stream(dev).wait_event(ev)


def _spec_stream(dev):
    # a library role stream (created once, low priority: the backward is off the critical path
    # until backward(), while predict()'s decode is on it), not a torch pool stream, whose
    # hardware queue depends on how many pool streams the process handed out before
    st = _SPEC_STREAMS.get(str(dev))
    if st is None:
        st = _SPEC_STREAMS[str(dev)] = (torch.cuda.Stream(dev)
                                        if os.environ.get("MPR_SPEC_STREAM") == "pool"
                                        else _lib.role_stream(dev, "train:spec"))
    return st


_TRAINERS = {}
# The native trainer's initial relative-position LUT radius (t5.LUT_RADIUS when None); its LUTs
# grow past it on demand (trainer.hip grow_luts).  The attention kernels take sequences of up to
# 1024 keys (max_source_length 512 + 50 image tokens is 562).
LUT_RADIUS_INIT = None


class T5Config:
    def __init__(self, names, shapes, num_heads, max_distance=128, scale_out=True):
        self.n_enc = _layers(names, "encoder")
        self.n_dec = _layers(names, "decoder")
        self.vocab, self.d = shapes["shared.weight"]
        self.num_buckets, self.H = shapes[
            "encoder.block.0.layer.0.SelfAttention.relative_attention_bias.weight"]
        assert self.H == num_heads
        self.inner = shapes["encoder.block.0.layer.0.SelfAttention.q.weight"][0]
        self.d_ff = shapes["encoder.block.0.layer.1.DenseReluDense.wi.weight"][0]
        self.max_distance = max_distance
        self.scale_out = scale_out
        self.dropout = None  # Dropout in train mode
        self.grad_enabled = True  # torch.is_grad_enabled() where the loss was built (t5_loss)

    def trainer(self, device):
        """The native trainer of this configuration on ``device`` (one per process; its tapes
        and scratch are reused step to step)."""
        cfg = (self.d, self.inner // self.H, self.H, self.d_ff, self.n_enc, self.n_dec,
               self.vocab, self.num_buckets, 1 if self.scale_out else 0)
        from .t5 import LUT_RADIUS
        radius = int(LUT_RADIUS_INIT or LUT_RADIUS)
        key = (cfg, self.max_distance, str(device), radius)
        tr = _TRAINERS.get(key)
        if tr is None:
            rel = torch.arange(-radius, radius + 1, dtype=torch.long)
            luts = [relative_position_bucket(rel, bi, self.num_buckets, self.max_distance)
                    for bi in (True, False)]
            tr = _lib.ctypes.c_void_p()
            _lib.call("mpr_t5_trainer_create", _lib.int_array(cfg), len(cfg),
                      _lib.int_array(luts[0].tolist()), _lib.int_array(luts[1].tolist()),
                      radius, _lib.ctypes.byref(tr))
            _TRAINERS[key] = tr
        return tr


def trim_trainers(keep_idle: int = 0, destroy: bool = False):
    """Hand the native trainers' device memory back (their tape arenas and scratch
    live outside torch's caching allocator, at their high-water mark): free the arenas of
    released tapes past the first ``keep_idle`` (mpr_t5_trainer_trim, after each device's
    queued work); ``destroy`` drops the trainers themselves (rebuilt on the next forward)."""
    for key, tr in list(_TRAINERS.items()):
        dev = torch.device(key[2])
        if destroy:
            torch.cuda.synchronize(dev)
            _lib.load().mpr_model_destroy(tr)
            del _TRAINERS[key]
            _LAST_SPEC.pop(tr.value, None)
        else:
            _after_spec(tr, dev)
            _lib.call("mpr_t5_trainer_trim", tr, int(keep_idle), _lib.stream_ptr(dev))


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
    cfg.grad_enabled = torch.is_grad_enabled()  # (off inside Function.forward)
    return T5LossFn.apply(cfg, inputs_embeds, attention_mask, labels,
                          *[named_params[n] for n in order])
