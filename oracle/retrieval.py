"""Oracle: retrieval scan, top-k and prompt construction (TEST INFRASTRUCTURE ONLY).

Restates dataset/VQAFeatureDataset.py:187-246 (VQADataset.retrieve_closest_qa_pairs) and
utils.py:57-62 (cosine_similarity).  Exact ties are ordered by lowest row id (the reference's
torch.argsort is unstable on ties; the build defines stable order).
"""
from __future__ import annotations

import numpy as np
import torch

BUCKETS = ["very unlikely", "unlikely", "maybe", "likely", "very likely", "certainly"]


def cdist(q: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """dataset/VQAFeatureDataset.py:192 — torch.cdist (Euclidean; mm path for > 25 rows)."""
    return torch.cdist(q.float(), x.float())


def topk_ids(dist: torch.Tensor, k: int, skip_first: bool) -> torch.Tensor:
    """dataset/VQAFeatureDataset.py:194-197 — argsort ascending, slice [s:s+k] (stable)."""
    order = torch.argsort(dist, dim=1, stable=True)
    s = 1 if skip_first else 0
    return order[:, s:s + k]


def vote_prompt(row_answers: list, use_quantifier: bool = True) -> str:
    """dataset/VQAFeatureDataset.py:216-230 — majority vote (first-inserted wins ties) and bucket."""
    counts: dict = {}
    for a in row_answers:
        counts[a] = counts.get(a, 0) + 1
    pred = max(counts, key=counts.get)
    certainty = max(counts.values()) / sum(counts.values())
    bucket = BUCKETS[int(certainty * (len(BUCKETS) - 1))]
    if use_quantifier:
        return f"I believe the answer is {bucket} {pred}"
    return f"The most frequent answer is {pred}"


def retrieve_closest_qa_pairs(query: torch.Tensor, index: torch.Tensor, answers: list,
                              question_info: dict, k: int, is_training_phase: bool,
                              return_ans=False, return_info=None, return_dists=False,
                              use_quantifier=True):
    """dataset/VQAFeatureDataset.py:187-246 given the already-encoded query [B, D]."""
    dist = cdist(query, index)
    ids = topk_ids(dist, k, is_training_phase)
    rows = [[answers[int(j)] for j in ids[i]] for i in range(ids.shape[0])]
    info = []
    if return_info:
        for r in ids:
            blk = []
            for j in r:
                for entry in return_info:
                    blk.append(question_info[entry][int(j)])
            info.append(blk)
    prompts = [vote_prompt(r, use_quantifier) for r in rows]
    if return_ans:
        return rows
    if return_info:
        return info
    if return_dists:
        smallest = torch.sort(dist, dim=1).values.numpy()[:, 0:k]
        return list(zip(rows, smallest))
    return prompts


def cosine_similarity(x1: torch.Tensor, x2: torch.Tensor, dim: int = 1, eps: float = 1e-8):
    """utils.py:57-62."""
    w12 = torch.sum(x1 * x2, dim)
    w1 = torch.norm(x1, 2, dim)
    w2 = torch.norm(x2, 2, dim)
    return (w12 / (w1 * w2).clamp(min=eps)).squeeze()


def cosine_topk(query: torch.Tensor, index: torch.Tensor, k: int):
    """Cosine-metric top-k (descending similarity, lowest id on ties) built on cosine_similarity."""
    sim = cosine_similarity(query[:, None, :], index[None, :, :], dim=2)
    if sim.dim() == 1:
        sim = sim[None]
    order = torch.from_numpy(np.lexsort((np.arange(sim.shape[1])[None].repeat(sim.shape[0], 0),
                                         -sim.numpy()), axis=1))
    ids = order[:, :k]
    return ids, torch.gather(sim, 1, ids)
