"""Oracle: CLIP ViT-B/32 image tower and CLIP text tower (TEST INFRASTRUCTURE ONLY).

Restates the openai CLIP arithmetic the reference calls (third-party, unpinned):
* ``encode_image`` — dataset/VQAFeatureDataset.py:146,189 (CLS -> ln_post -> @proj)
* ``get_image_token_features`` — architectures/T5VisionModel.py:112-139 (ln_post on ALL tokens)
* ``encode_text`` — dataset/VQAFeatureDataset.py:147,190 (causal, EOT = argmax(token id))
over openai-CLIP-named state dicts.  torch-CPU fp32 eager.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

LN_EPS = 1e-5


def _ln(x, sd, p):
    return F.layer_norm(x, (x.shape[-1],), sd[p + ".weight"], sd[p + ".bias"], LN_EPS)


def residual_block(x: torch.Tensor, sd: dict, p: str, heads: int, causal: bool) -> torch.Tensor:
    """openai CLIP ResidualAttentionBlock on x [B, L, W] (batch-first restatement)."""
    B, L, W = x.shape
    hd = W // heads
    h = _ln(x, sd, p + ".ln_1")
    qkv = h @ sd[p + ".attn.in_proj_weight"].T + sd[p + ".attn.in_proj_bias"]
    q, k, v = qkv.split(W, dim=-1)
    q = q.reshape(B, L, heads, hd).transpose(1, 2)
    k = k.reshape(B, L, heads, hd).transpose(1, 2)
    v = v.reshape(B, L, heads, hd).transpose(1, 2)
    s = (q @ k.transpose(-1, -2)) * (hd ** -0.5)
    if causal:
        s = s + torch.full((L, L), float("-inf")).triu_(1)
    a = torch.softmax(s, dim=-1) @ v
    a = a.transpose(1, 2).reshape(B, L, W)
    x = x + (a @ sd[p + ".attn.out_proj.weight"].T + sd[p + ".attn.out_proj.bias"])
    h = _ln(x, sd, p + ".ln_2")
    m = h @ sd[p + ".mlp.c_fc.weight"].T + sd[p + ".mlp.c_fc.bias"]
    m = m * torch.sigmoid(1.702 * m)
    return x + (m @ sd[p + ".mlp.c_proj.weight"].T + sd[p + ".mlp.c_proj.bias"])


def _layers(sd, prefix):
    n = 0
    while f"{prefix}.resblocks.{n}.ln_1.weight" in sd:
        n += 1
    return n


def vit_tokens(sd: dict, img: torch.Tensor) -> torch.Tensor:
    """Transformer output before ln_post: [B, g*g+1, W]."""
    w = sd["visual.conv1.weight"]
    W, p = w.shape[0], w.shape[-1]
    x = F.conv2d(img.float(), w, stride=p)                     # [B, W, g, g]
    x = x.reshape(x.shape[0], W, -1).permute(0, 2, 1)          # [B, g*g, W]
    cls = sd["visual.class_embedding"] + torch.zeros(x.shape[0], 1, W)
    x = torch.cat([cls, x], dim=1) + sd["visual.positional_embedding"]
    x = _ln(x, sd, "visual.ln_pre")
    heads = W // 64
    for i in range(_layers(sd, "visual.transformer")):
        x = residual_block(x, sd, f"visual.transformer.resblocks.{i}", heads, causal=False)
    return x


def encode_image(sd: dict, img: torch.Tensor) -> torch.Tensor:
    """CLIP.encode_image: [B, 512] from the CLS token."""
    x = vit_tokens(sd, img)
    return _ln(x[:, 0, :], sd, "visual.ln_post") @ sd["visual.proj"]


def image_token_features(sd: dict, img: torch.Tensor) -> torch.Tensor:
    """T5VisionModel.get_image_token_features: [B, 50, 512] (ln_post on every token)."""
    x = vit_tokens(sd, img)
    return _ln(x, sd, "visual.ln_post") @ sd["visual.proj"]


def encode_text(sd: dict, tokens: torch.Tensor) -> torch.Tensor:
    """CLIP.encode_text: tokens int [B, 77] -> [B, 512] at the EOT (argmax id) position."""
    tokens = tokens.long()
    x = sd["token_embedding.weight"][tokens] + sd["positional_embedding"]
    W = x.shape[-1]
    heads = W // 64
    for i in range(_layers(sd, "transformer")):
        x = residual_block(x, sd, f"transformer.resblocks.{i}", heads, causal=True)
    x = _ln(x, sd, "ln_final")
    x = x[torch.arange(x.shape[0]), tokens.argmax(dim=-1)]
    return x @ sd["text_projection"]
