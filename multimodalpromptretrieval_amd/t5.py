"""Device T5 (encoder, greedy generate, teacher-forced logits/loss) backed by libmpr.so.

Replaces the transformers T5ForConditionalGeneration calls of the reference:
``T5_model.shared(ids)`` (architectures/T5VisionModel.py:169), ``T5_model.generate(...)``
(:200-205) and ``T5_model(inputs_embeds, attention_mask, labels).loss`` (:233).
Weights are transformers-named state-dict tensors; relative-position bucket tables are computed
here on the host with the exact float32 expression of T5Attention._relative_position_bucket and
handed to the library once.
"""
from __future__ import annotations

import ctypes
import math
import os

import numpy as np
import torch

from . import _lib

LUT_RADIUS = 1024  # covers encoder lengths up to 512 and any decode length here
MAX_PIECES = 16    # batches of <= 16 rows sharing one decode loop (T5Model::MAX_GROUPS)


def pieces_per_call() -> int:
    """<= 16-row pieces per decode loop for a batch of more than 16 rows (predict() of a large
    batch, the serving loop's large batches): MPR_GEN_PIECES, default 16 (one 256-row loop for a
    256-question batch, every decode weight streamed once per step for all rows)."""
    return max(1, min(MAX_PIECES, int(os.environ.get("MPR_GEN_PIECES", "16"))))


def length_pieces(embeds, mask, lens=None):
    """A batch of more than 16 rows as 16-row pieces: (order, pieces).  With the rows' real
    lengths (``lens``, host ints: the leading ones of each right-padded mask row, e.g. the
    tokenizer's attention_mask sums) the rows go by length (stable) and each piece keeps only its
    own longest row's columns: the encoder then computes ~mean-length rows instead of the batch's
    longest (config C5: 62-71 % of a 256-question batch's padded rows are real tokens).  A row's
    result does not depend on its piece (every GEMM tile sums in the same order; columns past a
    row's length are masked keys, which add exact zeros), so the tokens come back in the caller's
    row order equal to the unsorted pieces'.  order None: the pieces are the rows in order."""
    B = embeds.shape[0]
    if lens is None or B <= 16:
        return None, [(embeds[i:i + 16], mask[i:i + 16]) for i in range(0, max(B, 1), 16)]
    lens = np.asarray(lens, dtype=np.int64).reshape(-1)
    if lens.shape[0] != B:
        raise ValueError(f"length_pieces: {lens.shape[0]} lengths for {B} rows")
    order = np.argsort(lens, kind="stable")
    idx = _lib.to_device_async(torch.from_numpy(order), embeds.device)
    e, m = embeds.index_select(0, idx), mask.index_select(0, idx)
    pieces = []
    for i in range(0, B, 16):
        lp = int(max(1, lens[order[i:i + 16]].max()))
        pieces.append((e[i:i + 16, :lp], m[i:i + 16, :lp]))
    return order, pieces


def relative_position_bucket(rel: torch.Tensor, bidirectional: bool, num_buckets: int = 32,
                             max_distance: int = 128) -> torch.Tensor:
    """T5Attention._relative_position_bucket (host-side integer metadata)."""
    buckets = torch.zeros_like(rel)
    if bidirectional:
        num_buckets //= 2
        buckets += (rel > 0).to(torch.long) * num_buckets
        rel = torch.abs(rel)
    else:
        rel = -torch.min(rel, torch.zeros_like(rel))
    max_exact = num_buckets // 2
    is_small = rel < max_exact
    large = max_exact + (torch.log(rel.float() / max_exact) / math.log(max_distance / max_exact)
                         * (num_buckets - max_exact)).to(torch.long)
    large = torch.min(large, torch.full_like(large, num_buckets - 1))
    return buckets + torch.where(is_small, rel, large)


def _layers(sd: dict, stack: str) -> int:
    n = 0
    while f"{stack}.block.{n}.layer.0.layer_norm.weight" in sd:
        n += 1
    return n


class DeviceT5:
    """T5ForConditionalGeneration arithmetic on one GPU (handle into libmpr)."""

    # generate() (predict()) decodes on workspace slots of its own (4, and 5 for more than 128
    # rows): a serving loop's calls in flight on slots 0-3 never block it, and it never blocks
    # them
    PREDICT_SLOT = 4

    def __init__(self, sd: dict, device, scale_decoder_outputs: bool = True,
                 max_distance: int = 128):
        _lib.ensure_device(device)
        self.device = torch.device(device)
        self.scale_out = scale_decoder_outputs
        self._h = None
        self._seen = {}
        shared = sd["shared.weight"]
        self.vocab, self.d_model = shared.shape
        q0 = sd["encoder.block.0.layer.0.SelfAttention.q.weight"]
        rel = sd["encoder.block.0.layer.0.SelfAttention.relative_attention_bias.weight"]
        self.num_buckets, self.num_heads = rel.shape
        self.inner = q0.shape[0]
        self.d_kv = self.inner // self.num_heads
        self.d_ff = sd["encoder.block.0.layer.1.DenseReluDense.wi.weight"].shape[0]
        self.n_enc = _layers(sd, "encoder")
        self.n_dec = _layers(sd, "decoder")
        self._max_distance = max_distance
        host, enc_lut, dec_lut = self._tensors(sd)
        cfg = [self.d_model, self.d_kv, self.num_heads, self.d_ff, self.n_enc, self.n_dec,
               self.vocab, self.num_buckets, 1 if scale_decoder_outputs else 0]
        h = _lib.ctypes.c_void_p()
        _lib.call("mpr_t5_create", _lib.int_array(cfg), len(cfg), _lib.tensor_array(host),
                  len(host), enc_lut, dec_lut, LUT_RADIUS, _lib.ctypes.byref(h))
        self._h = h

    def _tensors(self, sd: dict):
        """The mpr_t5_create tensor list of a transformers-named state dict + the bucket LUTs."""
        shared = sd["shared.weight"]
        rel = sd["encoder.block.0.layer.0.SelfAttention.relative_attention_bias.weight"]
        lm_head = sd.get("lm_head.weight", shared)
        t = [shared, rel]
        for i in range(self.n_enc):
            p = f"encoder.block.{i}.layer"
            t += [sd[p + ".0.layer_norm.weight"], sd[p + ".0.SelfAttention.q.weight"],
                  sd[p + ".0.SelfAttention.k.weight"], sd[p + ".0.SelfAttention.v.weight"],
                  sd[p + ".0.SelfAttention.o.weight"], sd[p + ".1.layer_norm.weight"],
                  sd[p + ".1.DenseReluDense.wi.weight"], sd[p + ".1.DenseReluDense.wo.weight"]]
        t += [sd["encoder.final_layer_norm.weight"],
              sd["decoder.block.0.layer.0.SelfAttention.relative_attention_bias.weight"]]
        for i in range(self.n_dec):
            p = f"decoder.block.{i}.layer"
            t += [sd[p + ".0.layer_norm.weight"], sd[p + ".0.SelfAttention.q.weight"],
                  sd[p + ".0.SelfAttention.k.weight"], sd[p + ".0.SelfAttention.v.weight"],
                  sd[p + ".0.SelfAttention.o.weight"], sd[p + ".1.layer_norm.weight"],
                  sd[p + ".1.EncDecAttention.q.weight"], sd[p + ".1.EncDecAttention.k.weight"],
                  sd[p + ".1.EncDecAttention.v.weight"], sd[p + ".1.EncDecAttention.o.weight"],
                  sd[p + ".2.layer_norm.weight"], sd[p + ".2.DenseReluDense.wi.weight"],
                  sd[p + ".2.DenseReluDense.wo.weight"]]
        t += [sd["decoder.final_layer_norm.weight"], lm_head]
        host = [x.detach().to(torch.float32).contiguous() for x in t]  # host or device
        if not hasattr(self, "_luts"):
            rel_pos = torch.arange(-LUT_RADIUS, LUT_RADIUS + 1, dtype=torch.long)
            enc = relative_position_bucket(rel_pos, True, self.num_buckets, self._max_distance)
            dec = relative_position_bucket(rel_pos, False, self.num_buckets, self._max_distance)
            self._luts = (_lib.int_array(enc.tolist()), _lib.int_array(dec.tolist()))
        return host, self._luts[0], self._luts[1]

    def update(self, sd: dict) -> "DeviceT5":
        """New parameter values (same shapes) into this handle's buffers: its captured generate
        graphs stay valid — an optimizer step costs a copy, not a rebuild.  Parameters on this
        device (training, main.py:186-187): mpr_t5_update_async, enqueued on the current stream
        after every stream this handle has run on, without a host wait; host tensors:
        mpr_t5_update (waits for the device)."""
        host, enc_lut, dec_lut = self._tensors(sd)
        if all(t.device == self.device for t in host):
            cur = torch.cuda.current_stream(self.device)
            for st in self._seen.values():
                if st.cuda_stream != cur.cuda_stream:
                    cur.wait_stream(st)
            _lib.call("mpr_t5_update_async", self._h, _lib.tensor_array(host), len(host),
                      _lib.c_void_p(cur.cuda_stream))
            self._seen[cur.cuda_stream] = cur
            # later work of this handle on any other stream waits for the refresh (_stream)
            self._refresh = torch.cuda.Event()
            self._refresh.record(cur)
            self._refresh_waited = {cur.cuda_stream}
        else:
            _lib.call("mpr_t5_update", self._h, _lib.tensor_array(host), len(host), enc_lut,
                      dec_lut)
        return self

    def close(self):
        if self._h is not None and _lib._lib is not None:
            _lib.load().mpr_model_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stream(self):
        # streams this handle's work was enqueued on: update() orders itself after them, and
        # each of them waits (once) for the newest asynchronous refresh before its next call
        st = torch.cuda.current_stream(self.device)
        self._seen[st.cuda_stream] = st
        ev = getattr(self, "_refresh", None)
        if ev is not None and st.cuda_stream not in self._refresh_waited:
            st.wait_event(ev)
            self._refresh_waited.add(st.cuda_stream)
        return _lib.c_void_p(st.cuda_stream)

    def set_decode_stream(self, stream=None, slot: int = 0):
        """Run the greedy decode loop of later generate calls on ``stream`` (a torch stream,
        e.g. ``_lib.role_stream(device, "decode")``; None = the caller's stream).  Ordering is
        unchanged: the loop waits for the encoder on the caller's stream and the caller's stream
        waits for the tokens."""
        if not hasattr(self, "_dec_streams"):
            self._dec_streams = {}
        self._dec_streams[slot] = stream  # keep the stream alive while the library uses it
        _lib.call("mpr_t5_set_decode_stream", self._h, int(slot),
                  _lib.c_void_p(stream.cuda_stream if stream is not None else 0))

    def embed(self, ids: torch.Tensor, out: torch.Tensor, row0: int = 0) -> torch.Tensor:
        """out[b, row0 + t, :] = shared[ids[b, t]] (out: [B, L, d] fp32 on device)."""
        ids32 = _lib.to_device_async(ids, self.device, torch.int32).contiguous()
        B, n = ids32.shape
        _lib.call("mpr_t5_embed", self._h, _lib.ptr(ids32), B, n, _lib.ptr(out),
                  out.shape[1] * out.shape[2], row0, self._stream())
        return out

    def _inputs(self, embeds, mask):
        embeds = embeds.to(self.device, torch.float32).contiguous()
        mask = mask.to(self.device, torch.float32).contiguous()
        if embeds.shape[-1] != self.d_model:
            raise RuntimeError(f"inputs_embeds width {embeds.shape[-1]} != d_model "
                               f"{self.d_model}")
        if mask.shape != embeds.shape[:2]:
            raise RuntimeError(f"attention_mask {tuple(mask.shape)} != {tuple(embeds.shape[:2])}")
        return embeds, mask

    def encode(self, embeds: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
        embeds, mask = self._inputs(embeds, mask)
        B, L, _ = embeds.shape
        out = torch.empty_like(embeds)
        _lib.call("mpr_t5_encode", self._h, _lib.ptr(embeds), _lib.ptr(mask), B, L,
                  _lib.ptr(out), self._stream())
        return out

    def generate_padded(self, embeds, mask, max_new_tokens=20, decoder_start_token_id=0,
                        eos_token_id=1, pad_token_id=0, slot: int = 0,
                        lens=None) -> torch.Tensor:
        """All max_new_tokens greedy steps on device: int32 [B, 1+max_new] (no host sync).
        ``slot`` picks one of the model's independent workspaces (two batches of a serving
        loop decode concurrently on different slots and streams).  A batch of more than 16 rows
        runs as 16-row chunks sharing decode loops (pieces_per_call() chunks per loop); with the
        rows' real lengths (``lens``) the chunks are length-ordered and trimmed
        (``length_pieces``)."""
        embeds, mask = self._inputs(embeds, mask)
        B, L, _ = embeds.shape
        if B > 16:
            order, chunks = length_pieces(embeds, mask, lens)
            if order is not None:
                toks = self.generate_padded_pieces(chunks, max_new_tokens, decoder_start_token_id,
                                                   eos_token_id, pad_token_id, slot)
                out = torch.empty_like(toks)
                out.index_copy_(0, _lib.to_device_async(torch.from_numpy(order), self.device),
                                toks)
                return out
            return self.generate_padded_pieces(chunks, max_new_tokens, decoder_start_token_id,
                                               eos_token_id, pad_token_id, slot)
        out = torch.empty((B, max_new_tokens + 1), device=self.device, dtype=torch.int32)
        _lib.call("mpr_t5_generate_slot", self._h, int(slot), _lib.ptr(embeds), _lib.ptr(mask),
                  B, L, int(max_new_tokens), int(decoder_start_token_id), int(eos_token_id),
                  int(pad_token_id), _lib.ptr(out), self._stream())
        return out

    def generate_padded_pieces(self, chunks, max_new_tokens=20, decoder_start_token_id=0,
                               eos_token_id=1, pad_token_id=0, slot: int = 0) -> torch.Tensor:
        """generate_padded over 16-row pieces [(embeds, mask), ...]: their tokens stacked."""
        per = pieces_per_call()
        groups = [chunks[g:g + per] for g in range(0, len(chunks), per)]
        outs = []
        if len(groups) == 1 or os.environ.get("MPR_SPLIT_SLOTS", "1") == "0":
            for grp in groups:
                outs += self.generate_batches_padded(grp, max_new_tokens,
                                                     decoder_start_token_id, eos_token_id,
                                                     pad_token_id, slot)
            return torch.cat(outs)
        # more than 128 rows (config C5's 256 questions): the 128-row decode loops are
        # latency-bound chains of launches that leave CUs idle, so consecutive loops run on
        # two workspace slots and streams at once (each loop's rows bit-identical to a call
        # of its own; the caller's stream waits for both)
        cur = torch.cuda.current_stream(self.device)
        sts = [_lib.role_stream(self.device, f"gen:{j}" if slot < self.PREDICT_SLOT
                                else f"pgen:{j}") for j in range(2)]
        for st in sts:
            st.wait_stream(cur)
        for gi, grp in enumerate(groups):
            st = sts[gi % 2]
            for e, m in grp:
                e.record_stream(st)
                m.record_stream(st)
            with torch.cuda.stream(st):
                o = self.generate_batches_padded(grp, max_new_tokens, decoder_start_token_id,
                                                 eos_token_id, pad_token_id,
                                                 slot=slot + gi % 2)
            for t in o:
                t.record_stream(cur)
            outs += o
        for st in sts:
            cur.wait_stream(st)
        return torch.cat(outs)

    def generate_batches_padded(self, batches, max_new_tokens=20, decoder_start_token_id=0,
                                eos_token_id=1, pad_token_id=0, slot: int = 0):
        """generate_padded() of 1-16 batches [(embeds, mask), ...] (<= 16 rows each) with one
        shared decode loop (mpr_t5_generate_batches): a list of [B_i, 1+max_new] int32, each
        bit-identical to its own call."""
        if not 1 <= len(batches) <= MAX_PIECES:
            raise ValueError(f"generate_batches: {len(batches)} batches (1 to {MAX_PIECES})")
        ins = [self._inputs(e, m) for e, m in batches]
        for e, _ in ins:
            if e.shape[0] > 16:
                raise ValueError(f"generate_batches: a batch of {e.shape[0]} rows (at most 16)")
        outs = [torch.empty((e.shape[0], max_new_tokens + 1), device=self.device,
                            dtype=torch.int32) for e, _ in ins]
        _lib.call("mpr_t5_generate_batches", self._h, int(slot), len(ins),
                  _lib.tensor_array([e for e, _ in ins]), _lib.tensor_array([m for _, m in ins]),
                  _lib.int_array([e.shape[0] for e, _ in ins]),
                  _lib.int_array([e.shape[1] for e, _ in ins]), int(max_new_tokens),
                  int(decoder_start_token_id), int(eos_token_id), int(pad_token_id),
                  _lib.tensor_array(outs), self._stream())
        return outs

    def generate_begin(self, batches, max_new_tokens=20, slot: int = 0, stop_chunk: int = 4,
                       ahead: int = 2, decoder_start_token_id=0, eos_token_id=1,
                       pad_token_id=0):
        """Non-blocking grouped generate with greedy search's stop (mpr_t5_generate_begin): the
        encoders and the first ``ahead`` decode chunks of ``stop_chunk`` steps are enqueued on
        the current stream; ``generate_poll(slot)`` advances the call.  Returns the [B_i,
        1+max_new] int32 output tensors, valid on the current stream once a poll reports done
        (each equal to generate_batches_padded's)."""
        if not 1 <= len(batches) <= MAX_PIECES:
            raise ValueError(f"generate_begin: {len(batches)} batches (1 to {MAX_PIECES})")
        ins = [self._inputs(e, m) for e, m in batches]
        for e, _ in ins:
            if e.shape[0] > 16:
                raise ValueError(f"generate_begin: a batch of {e.shape[0]} rows (at most 16)")
        outs = [torch.empty((e.shape[0], max_new_tokens + 1), device=self.device,
                            dtype=torch.int32) for e, _ in ins]
        _lib.call("mpr_t5_generate_begin", self._h, int(slot), len(ins),
                  _lib.tensor_array([e for e, _ in ins]), _lib.tensor_array([m for _, m in ins]),
                  _lib.int_array([e.shape[0] for e, _ in ins]),
                  _lib.int_array([e.shape[1] for e, _ in ins]), int(max_new_tokens),
                  int(decoder_start_token_id), int(eos_token_id), int(pad_token_id),
                  int(stop_chunk), int(ahead), _lib.tensor_array(outs), self._stream())
        return outs

    def generate_poll(self, slot: int = 0, wait: bool = False):
        """(done, decode steps launched) of the slot's generate_begin call; never blocks unless
        ``wait``.  When done, the tokens are ordered before later work on the current stream."""
        done, steps = ctypes.c_int32(0), ctypes.c_int32(0)
        _lib.call("mpr_t5_generate_poll", self._h, int(slot), int(bool(wait)),
                  ctypes.byref(done), ctypes.byref(steps), self._stream())
        return bool(done.value), int(steps.value)

    def generate_pair_padded(self, embeds_a, mask_a, embeds_b, mask_b, max_new_tokens=20,
                             decoder_start_token_id=0, eos_token_id=1, pad_token_id=0,
                             slot: int = 0):
        """generate_padded() of two batches with one shared decode loop (mpr_t5_generate_pair):
        ([B_a, 1+max_new], [B_b, 1+max_new]) int32, each bit-identical to its own call."""
        ea, ma = self._inputs(embeds_a, mask_a)
        eb, mb = self._inputs(embeds_b, mask_b)
        (Ba, La, _), (Bb, Lb, _) = ea.shape, eb.shape
        if Ba > 16 or Bb > 16:
            raise ValueError(f"generate_pair: batches of {Ba} and {Bb} rows (at most 16 each)")
        oa = torch.empty((Ba, max_new_tokens + 1), device=self.device, dtype=torch.int32)
        ob = torch.empty((Bb, max_new_tokens + 1), device=self.device, dtype=torch.int32)
        _lib.call("mpr_t5_generate_pair", self._h, int(slot), _lib.ptr(ea), _lib.ptr(ma), Ba, La,
                  _lib.ptr(eb), _lib.ptr(mb), Bb, Lb, int(max_new_tokens),
                  int(decoder_start_token_id), int(eos_token_id), int(pad_token_id),
                  _lib.ptr(oa), _lib.ptr(ob), self._stream())
        return oa, ob

    @staticmethod
    def trim(tokens: torch.Tensor, eos_token_id: int = 1) -> torch.Tensor:
        """Cut the padded token matrix where GenerationMixin stops (all rows finished)."""
        tok = tokens.cpu().long()
        T = tok.shape[1] - 1
        hit = (tok[:, 1:] == eos_token_id)
        if T == 0 or not bool(hit.any(dim=1).all()):
            return tok
        first = hit.float().argmax(dim=1) + 1        # column of each row's first eos
        return tok[:, :int(first.max()) + 1]

    def generate(self, embeds, mask, max_new_tokens=20, decoder_start_token_id=0,
                 eos_token_id=1, pad_token_id=0, lens=None, while_running=None) -> torch.Tensor:
        """GenerationMixin.generate(do_sample=False) result (int64, host, trimmed).  Stops where
        greedy search stops: the decode runs in chunks of MPR_EOS_STOP_CHUNK steps (default 4:
        no cost measurable against one graph, git show f10742c:tools/eos_chunk_ab.py, where 2 cost ~0.07 ms;
        0 = one graph of all steps) and no chunk is launched once every row has emitted eos
        (mpr_t5_generate_stop; the skipped columns are pad, as the full loop writes).
        ``while_running``: a host callable run once the encoder and the first decode chunks are
        enqueued, before the host waits on them (generate_begin + generate_poll: the same
        launches as mpr_t5_generate_stop)."""
        chunk = int(os.environ.get("MPR_EOS_STOP_CHUNK", "4"))
        embeds_, mask_ = self._inputs(embeds, mask)
        B, L, _ = embeds_.shape
        if chunk <= 0 or B > 16 or max_new_tokens <= chunk:
            if while_running is not None:
                while_running()
            toks = self.generate_padded(embeds, mask, max_new_tokens, decoder_start_token_id,
                                        eos_token_id, pad_token_id, slot=self.PREDICT_SLOT,
                                        lens=lens)
            self.last_steps_run = int(max_new_tokens)
            return self.trim(toks, eos_token_id)
        if while_running is not None:
            out = self.generate_begin([(embeds_, mask_)], max_new_tokens, slot=self.PREDICT_SLOT,
                                      stop_chunk=chunk, ahead=2,
                                      decoder_start_token_id=decoder_start_token_id,
                                      eos_token_id=eos_token_id, pad_token_id=pad_token_id)[0]
            try:
                while_running()
            finally:
                _, steps = self.generate_poll(self.PREDICT_SLOT, wait=True)
            self.last_steps_run = steps
            return self.trim(out, eos_token_id)
        out = torch.empty((B, max_new_tokens + 1), device=self.device, dtype=torch.int32)
        steps = ctypes.c_int32(0)
        _lib.call("mpr_t5_generate_stop", self._h, self.PREDICT_SLOT, _lib.ptr(embeds_),
                  _lib.ptr(mask_), B, L,
                  int(max_new_tokens), int(decoder_start_token_id), int(eos_token_id),
                  int(pad_token_id), chunk, _lib.ptr(out), ctypes.byref(steps), self._stream())
        self.last_steps_run = int(steps.value)
        return self.trim(out, eos_token_id)

    def logits(self, embeds, mask, decoder_input_ids) -> torch.Tensor:
        embeds, mask = self._inputs(embeds, mask)
        B, L, _ = embeds.shape
        dec = _lib.to_device_async(decoder_input_ids, self.device, torch.int32).contiguous()
        T = dec.shape[1]
        out = torch.empty((B, T, self.vocab), device=self.device, dtype=torch.float32)
        _lib.call("mpr_t5_logits", self._h, _lib.ptr(embeds), _lib.ptr(mask), B, L,
                  _lib.ptr(dec), T, _lib.ptr(out), self._stream())
        return out

    def loss(self, logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        lab = _lib.to_device_async(labels, self.device, torch.int32).contiguous()
        lg = logits.contiguous()
        out = torch.empty((), device=self.device, dtype=torch.float32)
        _lib.call("mpr_cross_entropy", _lib.ptr(lg), _lib.ptr(lab), lab.numel(),
                  lg.shape[-1], _lib.ptr(out), self._stream())
        return out
