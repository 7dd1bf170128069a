"""Oracle: T5 encoder, decoder and greedy generation (TEST INFRASTRUCTURE ONLY).

Restates transformers ``T5ForConditionalGeneration`` as the reference drives it
(architectures/T5VisionModel.py:200-205 generate(inputs_embeds, attention_mask,
do_sample=False, max_new_tokens=20); :233 teacher-forced loss) over HF-named state dicts:
RMSNorm (T5LayerNorm), unscaled attention with the layer-0 relative position bias
(T5Attention._relative_position_bucket / compute_bias), ReLU FFN, final norm, tied lm_head
after * d_model**-0.5.  torch-CPU fp32 eager.
"""
from __future__ import annotations

import math

import torch


def relative_position_bucket(rel: torch.Tensor, bidirectional: bool, num_buckets: int = 32,
                             max_distance: int = 128) -> torch.Tensor:
    """T5Attention._relative_position_bucket (transformers modeling_t5.py)."""
    buckets = torch.zeros_like(rel)
    if bidirectional:
        num_buckets //= 2
        buckets += (rel > 0).to(torch.long) * num_buckets
        rel = torch.abs(rel)
    else:
        rel = -torch.min(rel, torch.zeros_like(rel))
    max_exact = num_buckets // 2
    is_small = rel < max_exact
    large = max_exact + (
        torch.log(rel.float() / max_exact) / math.log(max_distance / max_exact)
        * (num_buckets - max_exact)
    ).to(torch.long)
    large = torch.min(large, torch.full_like(large, num_buckets - 1))
    return buckets + torch.where(is_small, rel, large)


def bucket_lut(radius: int, bidirectional: bool, num_buckets=32, max_distance=128) -> torch.Tensor:
    """Bucket of relative position r = key - query for r in [-radius, radius] (index r+radius)."""
    rel = torch.arange(-radius, radius + 1, dtype=torch.long)
    return relative_position_bucket(rel, bidirectional, num_buckets, max_distance)


def _rms(x, w, eps=1e-6):
    var = x.pow(2).mean(-1, keepdim=True)
    return w * (x * torch.rsqrt(var + eps))


def _n_layers(sd, stack):
    n = 0
    while f"{stack}.block.{n}.layer.0.layer_norm.weight" in sd:
        n += 1
    return n


def _attn(sd, p, h_q, h_kv, bias, heads):
    B, Lq, _ = h_q.shape
    Lk = h_kv.shape[1]
    q = (h_q @ sd[p + ".q.weight"].T).reshape(B, Lq, heads, -1).transpose(1, 2)
    k = (h_kv @ sd[p + ".k.weight"].T).reshape(B, Lk, heads, -1).transpose(1, 2)
    v = (h_kv @ sd[p + ".v.weight"].T).reshape(B, Lk, heads, -1).transpose(1, 2)
    s = q @ k.transpose(-1, -2)
    if bias is not None:
        s = s + bias
    a = torch.softmax(s.float(), dim=-1) @ v
    a = a.transpose(1, 2).reshape(B, Lq, -1)
    return a @ sd[p + ".o.weight"].T


def _mask_bias(mask: torch.Tensor) -> torch.Tensor:
    m = mask.float()[:, None, None, :]
    return (1.0 - m) * torch.finfo(torch.float32).min


def _pos_bias(sd, stack, Lq, Lk, bidirectional, q0=0):
    table = sd[f"{stack}.block.0.layer.0.SelfAttention.relative_attention_bias.weight"]
    ctx = torch.arange(Lq, dtype=torch.long)[:, None] + q0
    mem = torch.arange(Lk, dtype=torch.long)[None, :]
    b = relative_position_bucket(mem - ctx, bidirectional, table.shape[0])
    return table[b].permute(2, 0, 1).unsqueeze(0)             # [1, H, Lq, Lk]


def encode(sd: dict, embeds: torch.Tensor, mask: torch.Tensor, heads: int) -> torch.Tensor:
    """T5Stack (encoder) on inputs_embeds [B, L, d] -> last_hidden_state."""
    x = embeds.float()
    L = x.shape[1]
    bias = _pos_bias(sd, "encoder", L, L, True) + _mask_bias(mask)
    for i in range(_n_layers(sd, "encoder")):
        p = f"encoder.block.{i}.layer"
        h = _rms(x, sd[p + ".0.layer_norm.weight"])
        x = x + _attn(sd, p + ".0.SelfAttention", h, h, bias, heads)
        h = _rms(x, sd[p + ".1.layer_norm.weight"])
        f = torch.relu(h @ sd[p + ".1.DenseReluDense.wi.weight"].T)
        x = x + f @ sd[p + ".1.DenseReluDense.wo.weight"].T
    return _rms(x, sd["encoder.final_layer_norm.weight"])


def decoder_logits(sd: dict, enc: torch.Tensor, mask: torch.Tensor, dec_in: torch.Tensor,
                   heads: int, scale_decoder_outputs: bool = True) -> torch.Tensor:
    """Decoder (teacher forced, causal) + tied head: dec_in [B, T] -> logits [B, T, V]."""
    x = sd["shared.weight"][dec_in.long()]
    T = x.shape[1]
    self_bias = _pos_bias(sd, "decoder", T, T, False)
    self_bias = self_bias + torch.full((T, T), torch.finfo(torch.float32).min).triu_(1)
    cross_bias = _mask_bias(mask)
    for i in range(_n_layers(sd, "decoder")):
        p = f"decoder.block.{i}.layer"
        h = _rms(x, sd[p + ".0.layer_norm.weight"])
        x = x + _attn(sd, p + ".0.SelfAttention", h, h, self_bias, heads)
        h = _rms(x, sd[p + ".1.layer_norm.weight"])
        x = x + _attn(sd, p + ".1.EncDecAttention", h, enc, cross_bias, heads)
        h = _rms(x, sd[p + ".2.layer_norm.weight"])
        f = torch.relu(h @ sd[p + ".2.DenseReluDense.wi.weight"].T)
        x = x + f @ sd[p + ".2.DenseReluDense.wo.weight"].T
    x = _rms(x, sd["decoder.final_layer_norm.weight"])
    if scale_decoder_outputs:
        x = x * (x.shape[-1] ** -0.5)
    return x @ sd["lm_head.weight"].T


def generate(sd: dict, embeds: torch.Tensor, mask: torch.Tensor, heads: int,
             max_new_tokens: int = 20, start: int = 0, eos: int = 1, pad: int = 0,
             forced_steps: bool = False):
    """GenerationMixin greedy search (do_sample=False).

    Returns (tokens [B, 1+T], step_logits list of [B, V]).  Stops when every row has emitted
    eos (unless forced_steps), rows already finished emit pad.
    """
    enc = encode(sd, embeds, mask, heads)
    B = enc.shape[0]
    toks = torch.full((B, 1), start, dtype=torch.long)
    unfinished = torch.ones(B, dtype=torch.long)
    step_logits = []
    for _ in range(max_new_tokens):
        lg = decoder_logits(sd, enc, mask, toks, heads)[:, -1, :]
        step_logits.append(lg)
        nxt = torch.argmax(lg, dim=-1)
        nxt = nxt * unfinished + pad * (1 - unfinished)
        toks = torch.cat([toks, nxt[:, None]], dim=1)
        unfinished = unfinished & (nxt != eos).long()
        if not forced_steps and int(unfinished.max()) == 0:
            break
    return toks, step_logits


def generate_cached(sd: dict, embeds: torch.Tensor, mask: torch.Tensor, heads: int,
                    max_new_tokens: int = 20, start: int = 0, eos: int = 1, pad: int = 0,
                    forced_steps: bool = False) -> torch.Tensor:
    """Greedy search with a KV cache (the path transformers' generate takes: one decoder
    position per step, cross-attention K/V projected once).  Same tokens as ``generate``; this
    is the timed CPU baseline of bench.py."""
    enc = encode(sd, embeds, mask, heads)
    B = enc.shape[0]
    n_dec = _n_layers(sd, "decoder")
    cross_bias = _mask_bias(mask)
    table = sd["decoder.block.0.layer.0.SelfAttention.relative_attention_bias.weight"]

    def split(x):
        return x.reshape(B, x.shape[1], heads, -1).transpose(1, 2)

    ck, cv = [], []
    for i in range(n_dec):
        p = f"decoder.block.{i}.layer.1.EncDecAttention"
        ck.append(split(enc @ sd[p + ".k.weight"].T))
        cv.append(split(enc @ sd[p + ".v.weight"].T))
    sk = [None] * n_dec
    sv = [None] * n_dec
    toks = torch.full((B, 1), start, dtype=torch.long)
    cur = toks[:, 0]
    unfinished = torch.ones(B, dtype=torch.long)
    for t in range(max_new_tokens):
        x = sd["shared.weight"][cur][:, None, :]
        rel = torch.arange(t + 1, dtype=torch.long) - t
        bias = table[relative_position_bucket(rel, False, table.shape[0])].T[None, :, None, :]
        for i in range(n_dec):
            p = f"decoder.block.{i}.layer"
            h = _rms(x, sd[p + ".0.layer_norm.weight"])
            a = p + ".0.SelfAttention"
            q = split(h @ sd[a + ".q.weight"].T)
            k = split(h @ sd[a + ".k.weight"].T)
            v = split(h @ sd[a + ".v.weight"].T)
            sk[i] = k if sk[i] is None else torch.cat([sk[i], k], 2)
            sv[i] = v if sv[i] is None else torch.cat([sv[i], v], 2)
            w = torch.softmax(q @ sk[i].transpose(-1, -2) + bias, dim=-1)
            o = (w @ sv[i]).transpose(1, 2).reshape(B, 1, -1)
            x = x + o @ sd[a + ".o.weight"].T
            h = _rms(x, sd[p + ".1.layer_norm.weight"])
            c = p + ".1.EncDecAttention"
            q = split(h @ sd[c + ".q.weight"].T)
            w = torch.softmax(q @ ck[i].transpose(-1, -2) + cross_bias, dim=-1)
            o = (w @ cv[i]).transpose(1, 2).reshape(B, 1, -1)
            x = x + o @ sd[c + ".o.weight"].T
            h = _rms(x, sd[p + ".2.layer_norm.weight"])
            f = torch.relu(h @ sd[p + ".2.DenseReluDense.wi.weight"].T)
            x = x + f @ sd[p + ".2.DenseReluDense.wo.weight"].T
        x = _rms(x, sd["decoder.final_layer_norm.weight"]) * (x.shape[-1] ** -0.5)
        lg = (x @ sd["lm_head.weight"].T)[:, 0, :]
        nxt = torch.argmax(lg, dim=-1)
        nxt = nxt * unfinished + pad * (1 - unfinished)
        toks = torch.cat([toks, nxt[:, None]], dim=1)
        unfinished = unfinished & (nxt != eos).long()
        cur = nxt
        if not forced_steps and int(unfinished.max()) == 0:
            break
    return toks


def lm_loss(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """CrossEntropyLoss(ignore_index=-100) over [B, T, V] logits (T5ForConditionalGeneration)."""
    return torch.nn.functional.cross_entropy(logits.reshape(-1, logits.shape[-1]),
                                             labels.reshape(-1), ignore_index=-100)


def shift_right(labels: torch.Tensor, start: int = 0, pad: int = 0) -> torch.Tensor:
    """T5PreTrainedModel._shift_right: decoder inputs from labels (-100 -> pad)."""
    out = torch.full_like(labels, pad)
    out[:, 1:] = labels[:, :-1]
    out[:, 0] = start
    return out.masked_fill(out == -100, pad)
