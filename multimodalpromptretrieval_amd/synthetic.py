"""Deterministic synthetic weights and inputs (numpy PCG64) for tests, bench and goldens.

No checkpoints are reachable offline, so every model runs on seeded random
weights of the reference architectures:

* ``clip_state_dict`` — openai CLIP ViT-B/32 (visual.* + text tower) under the exact
  ``state_dict`` names of ``clip.load("ViT-B/32")`` (the reference's ``vision_model`` /
  ``clip_model``, architectures/T5VisionModel.py:26, dataset/VQAFeatureDataset.py:25).
* ``t5_state_dict`` — transformers ``T5ForConditionalGeneration`` names (the reference's
  ``T5_model``, architectures/T5VisionModel.py:59-60; vocab resized to 32101 = 32100 + "[itk]").
* ``images`` / ``clip_tokens`` / ``t5_prompt_ids`` / ``index_rows`` — SURVEY.md §8(d) inputs.

Initialisation follows the published init scales of both models so activations stay in the
regime of trained weights (no overflow over 12 layers), with random LayerNorm affines so the
affine paths are exercised.
"""
from __future__ import annotations

import functools

from dataclasses import dataclass

import numpy as np
import torch


@dataclass(frozen=True)
class ClipConfig:
    """openai CLIP ViT-B/32 geometry."""

    width: int = 768
    layers: int = 12
    heads: int = 12
    patch: int = 32
    image_size: int = 224
    embed_dim: int = 512
    text_width: int = 512
    text_layers: int = 12
    text_heads: int = 8
    context_length: int = 77
    vocab: int = 49408

    @property
    def grid(self) -> int:
        return self.image_size // self.patch


@dataclass(frozen=True)
class T5Config:
    """t5-small geometry (transformers T5Config defaults of the hub checkpoint)."""

    d_model: int = 512
    d_kv: int = 64
    num_heads: int = 8
    d_ff: int = 2048
    num_layers: int = 6
    num_decoder_layers: int = 6
    vocab_size: int = 32101
    relative_attention_num_buckets: int = 32
    relative_attention_max_distance: int = 128
    layer_norm_epsilon: float = 1e-6


T5_BASE = T5Config(d_model=768, d_kv=64, num_heads=12, d_ff=3072, num_layers=12,
                   num_decoder_layers=12)
SOT, EOT = 49406, 49407


def _rng(seed: int) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64(seed))


def _normal(rng: np.random.Generator, shape, std: float) -> torch.Tensor:
    return torch.from_numpy(rng.standard_normal(shape, dtype=np.float32) * np.float32(std))


def _ln(rng, sd: dict, prefix: str, width: int) -> None:
    sd[prefix + ".weight"] = 1.0 + _normal(rng, (width,), 0.1)
    sd[prefix + ".bias"] = _normal(rng, (width,), 0.1)


def _clip_blocks(rng, sd: dict, prefix: str, width: int, layers: int) -> None:
    attn_std = width ** -0.5
    proj_std = attn_std * (2 * layers) ** -0.5
    fc_std = (2 * width) ** -0.5
    for i in range(layers):
        p = f"{prefix}.resblocks.{i}"
        _ln(rng, sd, p + ".ln_1", width)
        sd[p + ".attn.in_proj_weight"] = _normal(rng, (3 * width, width), attn_std)
        sd[p + ".attn.in_proj_bias"] = _normal(rng, (3 * width,), 0.02)
        sd[p + ".attn.out_proj.weight"] = _normal(rng, (width, width), proj_std)
        sd[p + ".attn.out_proj.bias"] = _normal(rng, (width,), 0.02)
        _ln(rng, sd, p + ".ln_2", width)
        sd[p + ".mlp.c_fc.weight"] = _normal(rng, (4 * width, width), fc_std)
        sd[p + ".mlp.c_fc.bias"] = _normal(rng, (4 * width,), 0.02)
        sd[p + ".mlp.c_proj.weight"] = _normal(rng, (width, 4 * width), proj_std)
        sd[p + ".mlp.c_proj.bias"] = _normal(rng, (width,), 0.02)


def clip_state_dict(seed: int, cfg: ClipConfig = ClipConfig()) -> dict:
    """openai-CLIP-named fp32 state dict (visual tower + text tower)."""
    rng = _rng(seed)
    sd: dict = {}
    w = cfg.width
    scale = w ** -0.5
    sd["visual.conv1.weight"] = _normal(rng, (w, 3, cfg.patch, cfg.patch),
                                        (3 * cfg.patch * cfg.patch) ** -0.5)
    sd["visual.class_embedding"] = _normal(rng, (w,), scale)
    sd["visual.positional_embedding"] = _normal(rng, (cfg.grid ** 2 + 1, w), scale)
    _ln(rng, sd, "visual.ln_pre", w)
    _clip_blocks(rng, sd, "visual.transformer", w, cfg.layers)
    _ln(rng, sd, "visual.ln_post", w)
    sd["visual.proj"] = _normal(rng, (w, cfg.embed_dim), scale)
    tw = cfg.text_width
    sd["token_embedding.weight"] = _normal(rng, (cfg.vocab, tw), 0.02)
    sd["positional_embedding"] = _normal(rng, (cfg.context_length, tw), 0.01)
    _clip_blocks(rng, sd, "transformer", tw, cfg.text_layers)
    _ln(rng, sd, "ln_final", tw)
    sd["text_projection"] = _normal(rng, (tw, cfg.embed_dim), tw ** -0.5)
    sd["logit_scale"] = torch.tensor(float(np.log(1 / 0.07)), dtype=torch.float32)
    return sd


def t5_state_dict(seed: int, cfg: T5Config = T5Config()) -> dict:
    """transformers-T5-named fp32 state dict (tied lm_head)."""
    rng = _rng(seed)
    d, dkv, H, dff = cfg.d_model, cfg.d_kv, cfg.num_heads, cfg.d_ff
    inner = H * dkv
    sd: dict = {}
    # A tied random T5 with unit-std embeddings just copies its input token forever; a small
    # embedding scale lets the layers steer the argmax, and a 2x eos row makes some rows stop
    # early, so greedy parity tests see varied tokens and the early-stop path.
    shared = _normal(rng, (cfg.vocab_size, d), 0.05)
    shared[1] *= 2.0
    sd["shared.weight"] = shared

    def attn(p, rel):
        sd[p + ".q.weight"] = _normal(rng, (inner, d), (d * dkv) ** -0.5)
        sd[p + ".k.weight"] = _normal(rng, (inner, d), d ** -0.5)
        sd[p + ".v.weight"] = _normal(rng, (inner, d), d ** -0.5)
        sd[p + ".o.weight"] = _normal(rng, (d, inner), inner ** -0.5)
        if rel:
            sd[p + ".relative_attention_bias.weight"] = _normal(
                rng, (cfg.relative_attention_num_buckets, H), d ** -0.5)

    def ln(p):
        sd[p + ".weight"] = 1.0 + _normal(rng, (d,), 0.1)

    def ffn(p):
        sd[p + ".DenseReluDense.wi.weight"] = _normal(rng, (dff, d), d ** -0.5)
        sd[p + ".DenseReluDense.wo.weight"] = _normal(rng, (d, dff), dff ** -0.5)

    for i in range(cfg.num_layers):
        p = f"encoder.block.{i}.layer"
        attn(p + ".0.SelfAttention", rel=(i == 0))
        ln(p + ".0.layer_norm")
        ffn(p + ".1")
        ln(p + ".1.layer_norm")
    ln("encoder.final_layer_norm")
    for i in range(cfg.num_decoder_layers):
        p = f"decoder.block.{i}.layer"
        attn(p + ".0.SelfAttention", rel=(i == 0))
        ln(p + ".0.layer_norm")
        attn(p + ".1.EncDecAttention", rel=False)
        ln(p + ".1.layer_norm")
        ffn(p + ".2")
        ln(p + ".2.layer_norm")
    ln("decoder.final_layer_norm")
    sd["encoder.embed_tokens.weight"] = shared
    sd["decoder.embed_tokens.weight"] = shared
    sd["lm_head.weight"] = shared
    return sd


def eos_early_t5(sd: dict) -> dict:
    """A T5 whose greedy search ends at step 1 in every row, as a trained SLAKE model's short
    answers end after a few tokens: decoder layers that add nothing (self-attention o, cross o and
    FFN wo zero) and a tied embedding whose eos row is 100 x the start token's, so the first step's
    argmax is eos everywhere."""
    sd = {k: v.clone() for k, v in sd.items()}
    for k in list(sd):
        if k.startswith("decoder.block.") and (k.endswith("SelfAttention.o.weight")
                                              or k.endswith("EncDecAttention.o.weight")
                                              or k.endswith("DenseReluDense.wo.weight")):
            sd[k].zero_()
    sd["shared.weight"][1] = 100.0 * sd["shared.weight"][0]
    for k in ("lm_head.weight", "encoder.embed_tokens.weight", "decoder.embed_tokens.weight"):
        if k in sd:
            sd[k] = sd["shared.weight"]
    return sd


def images(seed: int, b: int, size: int = 224) -> torch.Tensor:
    """CLIP-normalised-range images fp32 [b, 3, size, size]."""
    x = _rng(seed).standard_normal((b, 3, size, size), dtype=np.float32)
    return torch.from_numpy(np.clip(x, -1.8, 2.2))


def clip_tokens(seed: int, b: int, ctx: int = 77, lo: int = 8, hi: int = 24) -> torch.Tensor:
    """clip.tokenize-shaped ids int64 [b, ctx]: [SOT, words..., EOT, 0...], length U(lo, hi)."""
    rng = _rng(seed)
    out = np.zeros((b, ctx), dtype=np.int64)
    for i in range(b):
        n = int(rng.integers(lo, hi + 1))
        out[i, 0] = SOT
        out[i, 1:n - 1] = rng.integers(1, SOT, size=n - 2)
        out[i, n - 1] = EOT
    return torch.from_numpy(out)


def t5_prompt_ids(seed: int, b: int, lo: int = 15, hi: int = 30, vocab: int = 32100):
    """Right-padded T5 prompt ids [b, L] (+EOS=1) and attention mask, L = longest row."""
    rng = _rng(seed)
    lens = rng.integers(lo, hi + 1, size=b)
    L = int(lens.max())
    ids = np.zeros((b, L), dtype=np.int64)
    mask = np.zeros((b, L), dtype=np.int64)
    for i, n in enumerate(lens):
        ids[i, :n - 1] = rng.integers(2, vocab - 1, size=n - 1)
        ids[i, n - 1] = 1
        mask[i, :n] = 1
    return torch.from_numpy(ids), torch.from_numpy(mask)


def index_rows(seed: int, n: int, d: int, sigma: float = 0.3) -> torch.Tensor:
    """Retrieval index fp32 [n, d] = randn * sigma (CLIP-like row norms ~10 at d=1024)."""
    return _normal(_rng(seed), (n, d), sigma)


def index_rows_device(seed: int, lo: int, hi: int, d: int, device, sigma: float = 0.3,
                      chunk: int = 1 << 16) -> torch.Tensor:
    """Rows [lo, hi) of a large synthetic index generated on the device in fixed chunks of
    `chunk` rows (chunk c seeded with seed * 1_000_003 + c), so a row's content does not depend
    on how the index is sharded (C5: 1,048,576 x 512 split over 1/2/4/8 ranks)."""
    out = torch.empty((hi - lo, d), device=device, dtype=torch.float32)
    g = torch.Generator(device=device)
    c = lo // chunk
    while c * chunk < hi:
        a, b = max(lo, c * chunk), min(hi, (c + 1) * chunk)
        g.manual_seed(seed * 1_000_003 + c)
        full = torch.randn((chunk, d), device=device, generator=g) * sigma
        out[a - lo:b - lo] = full[a - c * chunk:b - c * chunk]
        c += 1
    return out


def answers(n: int, vocab: int = 50) -> list:
    return [f"a{j % vocab}" for j in range(n)]


# ---- offline tokenizers --------------------------------------------------------------------
# Neither the CLIP BPE vocab nor T5's spiece.model exist offline (SURVEY.md §7 hard part iv), so
# tests, goldens and the bench use deterministic word-hash tokenizers with the call surface the
# reference uses (clip.tokenize; T5Tokenizer.__call__/batch_decode/add_tokens/...).  Real
# tokenizers are used automatically when `clip` / the hub checkpoint are available.

@functools.lru_cache(maxsize=1 << 16)
def _fnv1a(word: str) -> int:
    # memoised: a stand-in for a compiled tokenizer should not cost Python loops per character
    # on every call (the real T5 / CLIP tokenizers are native code)
    h = 0x811C9DC5
    for ch in word.encode("utf-8"):
        h = ((h ^ ch) * 0x01000193) & 0xFFFFFFFF
    return h


def hash_clip_tokenize(texts, context_length: int = 77, truncate: bool = False) -> torch.Tensor:
    """clip.tokenize stand-in: [SOT, hash(word)..., EOT, 0...] int64 [B, context_length]."""
    if isinstance(texts, str):
        texts = [texts]
    out = torch.zeros(len(texts), context_length, dtype=torch.long)
    for i, t in enumerate(texts):
        ids = [SOT] + [1 + _fnv1a(w) % (SOT - 1) for w in t.lower().split()] + [EOT]
        if len(ids) > context_length:
            if not truncate:
                raise RuntimeError(f"Input {t} is too long for context length {context_length}")
            ids = ids[:context_length]
            ids[-1] = EOT
        out[i, :len(ids)] = torch.tensor(ids)
    return out


class HashT5Tokenizer:
    """T5Tokenizer stand-in: pad=0, eos=1, unk=2, words hashed into [3, 32100), added tokens
    appended after 32100 (so "[itk]" -> 32100 as in architectures/T5VisionModel.py:58-61)."""

    pad_token_id, eos_token_id, unk_token_id = 0, 1, 2
    base_vocab = 32100

    def __init__(self):
        self._added: dict = {}
        self._rev: dict = {0: "<pad>", 1: "</s>", 2: "<unk>"}

    def __len__(self):
        return self.base_vocab + len(self._added)

    def add_tokens(self, toks):
        n = 0
        for t in toks:
            if t not in self._added:
                self._added[t] = self.base_vocab + len(self._added)
                self._rev[self._added[t]] = t
                n += 1
        return n

    def convert_tokens_to_ids(self, tok):
        if tok in self._added:
            return self._added[tok]
        return self._word_id(tok)

    def _word_id(self, w: str) -> int:
        i = 3 + _fnv1a(w) % (self.base_vocab - 3)
        self._rev.setdefault(i, w)
        return i

    def encode_one(self, text: str, max_length=None, truncation=False) -> list:
        ids = [self._added.get(w, None) or self._word_id(w) for w in text.split()] + [1]
        if truncation and max_length is not None and len(ids) > max_length:
            ids = ids[:max_length - 1] + [1]
        return ids

    def __call__(self, texts, padding="longest", max_length=None, truncation=False,
                 return_tensors=None):
        from transformers import BatchEncoding
        if isinstance(texts, str):
            texts = [texts]
        rows = [self.encode_one(t, max_length, truncation) for t in texts]
        L = max(len(r) for r in rows) if padding else None
        ids, mask = [], []
        for r in rows:
            n = L if L is not None else len(r)
            ids.append(r + [self.pad_token_id] * (n - len(r)))
            mask.append([1] * len(r) + [0] * (n - len(r)))
        if return_tensors == "pt":
            return BatchEncoding({"input_ids": torch.tensor(ids, dtype=torch.long),
                                  "attention_mask": torch.tensor(mask, dtype=torch.long)})
        return BatchEncoding({"input_ids": ids, "attention_mask": mask})

    def convert_ids_to_tokens(self, ids):
        return [self._rev.get(int(i), f"<{int(i)}>") for i in ids]

    def batch_decode(self, seqs, skip_special_tokens=False):
        out = []
        for s in seqs:
            words = []
            for i in (s.tolist() if hasattr(s, "tolist") else s):
                i = int(i)
                if skip_special_tokens and i in (0, 1, 2):
                    continue
                words.append(self._rev.get(i, f"<{i}>"))
            out.append(" ".join(words))
        return out
