"""Seed-derived inputs of the golden fixtures (shared by make_goldens.py and the tests).

Nothing here imports the reference; the GPU box regenerates every input from these seeds.
"""
from __future__ import annotations

import numpy as np
import torch

from multimodalpromptretrieval_amd import synthetic as syn

# ---- G1: retrieval scan -------------------------------------------------------------------
G1_CASES = [(512, 512), (6500, 1024)]
G1_K = [1, 3, 5, 15]
G1_B = 16
G1_ANS_VOCAB = 7
TIE_DUPES = [17, 101, 250]
TIE_SOURCE = 200
TIE_QUERIES = [200, 5, 17, 101]


def g1_seed(N, D):
    return 100 + N + D


def g1_queries(N, D, seed):
    """Index [N, D] and 16 queries near index rows (self-matches for the training phase) at
    increasing noise, so both exact self-hits and genuinely nearest-neighbour cases occur."""
    X = syn.index_rows(seed, N, D)
    rng = np.random.Generator(np.random.PCG64(seed + 1000))
    rows = rng.choice(N, size=G1_B, replace=False)
    noise = syn.index_rows(seed + 2000, G1_B, D)
    scale = torch.tensor([0.0, 0.0, 0.0, 0.0, 0.01, 0.01, 0.05, 0.05, 0.1, 0.1, 0.3, 0.3,
                          1.0, 1.0, 3.0, 3.0])[:, None]
    q = X[rows] + noise * scale
    return X, q, rows


def question_info(N):
    return {"question_id": [str(j) for j in range(N)],
            "question_type": ["open" if j % 3 else "closed" for j in range(N)],
            "question": [f"q{j}" for j in range(N)]}


def tie_index():
    g = np.random.Generator(np.random.PCG64(5))
    X = torch.from_numpy(g.integers(-3, 4, size=(300, 64)).astype(np.float32))
    X[TIE_DUPES] = X[TIE_SOURCE].clone()
    return X, X[TIE_QUERIES].clone()


# ---- G2: tiny end-to-end pipeline (reference T5VisionModel + retrieval) ------------------------
G2 = {"clip_cfg": dict(width=128, layers=2, heads=2, patch=32, image_size=64, embed_dim=64,
                       text_width=128, text_layers=2, text_heads=2),
      "tok_cfg": dict(width=128, layers=2, heads=2, patch=32, image_size=64, embed_dim=128,
                      text_width=128, text_layers=1, text_heads=2),
      "t5_cfg": dict(d_model=128, d_kv=64, num_heads=2, d_ff=256, num_layers=2,
                     num_decoder_layers=2),
      "seeds": {"clip": 301, "tok": 302, "t5": 303, "index": 304, "images": 305},
      "N": 300, "B": 6, "k": 3, "index_sigma": 0.15, "ans_vocab": 5}


def g2_models():
    ccfg = syn.ClipConfig(**G2["clip_cfg"])
    tcfg = syn.ClipConfig(**G2["tok_cfg"])
    t5cfg = syn.T5Config(**G2["t5_cfg"])
    return (ccfg, syn.clip_state_dict(G2["seeds"]["clip"], ccfg),
            tcfg, syn.clip_state_dict(G2["seeds"]["tok"], tcfg),
            t5cfg, syn.t5_state_dict(G2["seeds"]["t5"], t5cfg))


def g2_index(ccfg):
    N = G2["N"]
    X = syn.index_rows(G2["seeds"]["index"], N, 2 * ccfg.embed_dim, sigma=G2["index_sigma"])
    return X, syn.answers(N, G2["ans_vocab"]), question_info(N)


def g2_batch():
    B = G2["B"]
    rng = np.random.Generator(np.random.PCG64(306))
    words = ["what", "is", "the", "organ", "shown", "in", "this", "image", "does", "picture",
             "contain", "lung", "liver", "brain", "which", "modality", "used", "where", "mass"]
    qs = [" ".join(rng.choice(words, size=int(rng.integers(4, 10)))) for _ in range(B)]
    tasks = [["organ", "modality", "position", "abnormality"][i % 4] for i in range(B)]
    answers = [["yes", "no", "lung", "liver cancer", "ct", "left lung"][i % 6] for i in range(B)]
    return {"image": syn.images(G2["seeds"]["images"], B, G2["clip_cfg"]["image_size"]),
            "question": qs, "task": tasks, "answer": answers,
            "question_id": [str(i) for i in range(B)], "question_type": ["open"] * B}


# ---- G3 / G4: full-size third-party arithmetic (transformers T5 / CLIP second source) ---------
G3 = {"t5_seed": 401, "ids_seed": 402, "img_seed": 403, "B": 4, "vocab_sel_seed": 404}
G4 = {"clip_seed": 501, "img_seed": 502, "tok_seed": 503, "B_img": 2, "B_txt": 3}


def g3_inputs(d_model=512):
    B = G3["B"]
    ids, tmask = syn.t5_prompt_ids(G3["ids_seed"], B)
    img_tok = syn._normal(syn._rng(G3["img_seed"]), (B, 50, d_model), 0.5)
    mask = torch.cat([torch.ones(B, 50, dtype=torch.long), tmask], 1)
    return ids, img_tok, mask


# ---- G5: utils.cosine_similarity (reference utils.py:57-62) ----------------------------------
G5 = {"seed": 601, "aligned": (16, 1024), "aligned3": (4, 8, 64), "pair_B": 16, "pair_N": 600,
      "pair_D": 1024}


def g5_inputs():
    """(name, x1, x2, dim) cases: aligned rows (dim 1 and a middle dim), a zero row (the eps
    clamp), the [B,1,D] x [1,N,D] retrieval-matrix pattern, and a single-query pairwise call
    (squeeze to [N])."""
    s = G5["seed"]
    B, D = G5["aligned"]
    a1, a2 = syn.index_rows(s, B, D), syn.index_rows(s + 1, B, D)
    a1[3] = 0.0
    t1, t2 = syn.index_rows(s + 2, 4 * 8, 64).view(4, 8, 64), \
        syn.index_rows(s + 3, 4 * 8, 64).view(4, 8, 64)
    pB, pN, pD = G5["pair_B"], G5["pair_N"], G5["pair_D"]
    q = syn.index_rows(s + 4, pB, pD)[:, None, :]
    X = syn.index_rows(s + 5, pN, pD)[None]
    return [("aligned", a1, a2, 1), ("aligned3_dim2", t1, t2, 2),
            ("aligned3_dim1", t1.transpose(1, 2).contiguous(), t2.transpose(1, 2).contiguous(), 1),
            ("pairwise", q, X, 2), ("pairwise_one", q[:1], X, 2)]


# ---- G6: retrieval off (config C1: retrieval_function=None, architectures/T5VisionModel.py:148)
# ---- G7: t5-base behind the reference model with use_image_info=0 (config C5) -------
G7 = {"t5_seed": 701}


# ---- G8: a source past 256 / 512 keys (50 image tokens + 512 text tokens, max_source_length) --
G8 = {"t5_seed": 801, "ids_seed": 802, "img_seed": 803, "B": 2, "L_txt": [512, 301]}


def g8_inputs(d_model=512):
    """Two rows: 50 image tokens + 512 text tokens (the longest source the reference can build,
    L = 562) and + 301 (padded)."""
    B = G8["B"]
    rng = syn._rng(G8["ids_seed"])
    L = max(G8["L_txt"])
    ids = torch.zeros((B, L), dtype=torch.long)
    tmask = torch.zeros((B, L), dtype=torch.long)
    for i, n in enumerate(G8["L_txt"]):
        ids[i, :n - 1] = torch.from_numpy(rng.integers(2, 32099, size=n - 1))
        ids[i, n - 1] = 1
        tmask[i, :n] = 1
    img_tok = syn._normal(syn._rng(G8["img_seed"]), (B, 50, d_model), 0.5)
    mask = torch.cat([torch.ones(B, 50, dtype=torch.long), tmask], 1)
    return ids, img_tok, mask


# ---- G9: main.py-shaped harness (create_retrieval_dataset over a loader, then per test batch
# ---- predict + the four analytics calls, main.py:119-123, 262-270) on the G2 models ----------
G9 = {"retr_batches": 4, "test_batches": 3, "B": 6, "k": 3, "seed": 901}
G9_ANSWERS = ["yes", "no", "lung", "liver", "ct", "mri", "left", "brain"]


def _g9_batch(seed, B, qid0):
    rng = np.random.Generator(np.random.PCG64(seed))
    words = ["what", "is", "the", "organ", "shown", "in", "this", "image", "does", "picture",
             "contain", "lung", "liver", "brain", "which", "modality", "used", "where", "mass"]
    return {"image": syn.images(seed, B, G2["clip_cfg"]["image_size"]),
            "question": [" ".join(rng.choice(words, size=int(rng.integers(4, 10))))
                         for _ in range(B)],
            "task": [["organ", "modality", "position", "abnormality"][int(t)]
                     for t in rng.integers(0, 4, size=B)],
            "answer": [G9_ANSWERS[int(a)] for a in rng.integers(0, len(G9_ANSWERS), size=B)],
            "question_id": [str(qid0 + i) for i in range(B)],
            "question_type": [["open", "closed"][int(t)] for t in rng.integers(0, 2, size=B)]}


def g9_retrieval_loader():
    return [_g9_batch(G9["seed"] + i, G9["B"], 1000 + i * G9["B"])
            for i in range(G9["retr_batches"])]


def g9_test_batches():
    return [_g9_batch(G9["seed"] + 100 + i, G9["B"], 5000 + i * G9["B"])
            for i in range(G9["test_batches"])]


# ---- G10 / G11: training gradients (main.py:177-188) -----------------
# G10: the reference's own T5VisionModel.forward(batch).backward() at G2 size (all T5 gradients;
# the [32101, 128] shared gradient as its norm plus a row sample).  G11: transformers
# T5ForConditionalGeneration at full t5-small size on the G3 inputs with labels below (per
# parameter: gradient norm + its first 256 values; shared: norm + row sample).
G10 = {"rows_seed": 1001, "n_rows": 192}
G11 = {"t5_seed": 1101, "lab_seed": 1102, "T": 7, "rows_seed": 1103, "n_rows": 96}
G12 = {"p": 0.1, "seed": 1201}  # train-mode dropout (make_g12)


def g11_labels(B: int):
    """[B, T] label ids (1..999, eos 1 at each row's end, -100 after it)."""
    rng = np.random.Generator(np.random.PCG64(G11["lab_seed"]))
    T = G11["T"]
    lab = torch.tensor(rng.integers(2, 1000, size=(B, T)), dtype=torch.long)
    for b in range(B):
        n = 2 + b % (T - 1)
        lab[b, n - 1] = 1
        lab[b, n:] = -100
    return lab


def shared_rows(seed: int, n: int, vocab: int, must):
    """sorted(rows the batch touches ∪ n random rows) of the shared gradient to compare."""
    rng = np.random.Generator(np.random.PCG64(seed))
    rows = set(int(x) for x in must) | set(int(x) for x in rng.choice(vocab, n, replace=False))
    return np.array(sorted(r for r in rows if 0 <= r < vocab), dtype=np.int64)
