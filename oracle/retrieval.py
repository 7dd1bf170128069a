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


def smallest_dists(query: torch.Tensor, index: torch.Tensor, k: int) -> torch.Tensor:
    """dataset/VQAFeatureDataset.py:242-245 — the `return_dists` values: the k smallest cdist
    entries per row, [B, k] fp32 (the training phase does not skip the self match here)."""
    return torch.sort(cdist(query, index), dim=1).values[:, 0:k]


def rank_margins(query: torch.Tensor, index: torch.Tensor, k: int, skip_first: bool):
    """SURVEY.md §7 hard part (i): per query, the fp64 squared-distance gap between the last
    retrieved rank and the first one left out (ranks s+k-1 and s+k, s = 1 in the training
    phase), absolute and relative to |q|^2 + |x|^2 of those rows.  A retrieved-id set can only
    change under a perturbation of the query or of the summation order that moves a squared
    distance by more than half that gap.  Returns (gap [B], rel_gap [B], fp64 |q - x_last| [B]);
    inf where the index has no row past the retrieved ones."""
    qd, xd = query.double(), index.double()
    d2 = (qd * qd).sum(1, keepdim=True) + (xd * xd).sum(1)[None, :] - 2.0 * qd @ xd.T
    s = 1 if skip_first else 0
    last = s + k - 1
    B, n = d2.shape
    if last + 1 >= n:
        inf = torch.full((B,), float("inf"), dtype=torch.float64)
        return inf, inf, d2.clamp(min=0).sqrt().max(1).values
    v, i = torch.topk(d2, last + 2, dim=1, largest=False, sorted=True)
    gap = v[:, last + 1] - v[:, last]
    scale = (qd * qd).sum(1) + (xd * xd).sum(1)[i[:, last]]
    return gap, gap / scale, v[:, last].clamp(min=0).sqrt()


def id_parity(ids, dists, query, trace: dict) -> dict:
    """Checker for a device retrieval against ``pipeline.predict(..., trace=...)`` on the same
    batch: ``ids`` [B, k] (the retrieved example ids, e.g. ``return_info=["question_id"]``),
    ``dists`` [B, k] (``return_dists``), ``query`` [B, D] the device's query rows.

    The device query comes from fp32-accurate device towers, the oracle's from torch-CPU fp32,
    so the two differ by |dq| (measured here).  Squared distances then differ by at most
    2|dq|·|q - x| + |dq|^2 plus the mm-path evaluation error 2e-6·(|q|^2 + |x|^2) (§4 of
    DESIGN.md), and a retrieved id can differ only where the fp64 rank margin (``rank_margins``)
    is below twice that.  Returns counts and the worst margins (plain Python values)."""
    ids = torch.as_tensor(np.asarray(ids), dtype=torch.int64)
    got = torch.as_tensor(np.asarray(dists), dtype=torch.float64)
    want_ids, want = trace["ids"].to(torch.int64), trace["dists"].double()
    qo = trace["query"].double()
    dq = (torch.as_tensor(query).double().cpu() - qo).norm(dim=1)          # [B]
    qn = (qo * qo).sum(1)
    d_last = trace["d_last"]
    gap = trace["gap"]
    d_next = torch.where(torch.isfinite(gap), (d_last * d_last + gap).sqrt(), d_last)
    pert = 2.0 * dq * d_next + dq * dq                  # [B]: |d2(q + dq) - d2(q)|, any kept row
    scale = qn + (qn.sqrt() + d_next) ** 2               # >= |q|^2 + |x|^2, ranks 1 .. k+1
    tol2 = 2e-6 * scale + pert
    derr = (got * got - want * want).abs().amax(1)
    rows_equal = (ids == want_ids).all(1)
    # >= 1: the rank k / k+1 gap exceeds what both the query difference and the two sides'
    # fp32 evaluation errors can move, so equal ids are implied, not luck
    guard = gap / (2.0 * (pert + 2e-6 * scale))
    return {"rows": int(ids.shape[0]), "ids_equal_rows": int(rows_equal.sum()),
            "ids_equal": bool(rows_equal.all()),
            "dists_within_bound": bool((derr <= tol2).all()),
            "max_dist2_err_over_bound": float((derr / tol2).max()),
            "max_query_delta": float(dq.max()),
            "max_query_delta_rel": float((dq / qn.sqrt()).max()),
            "min_rel_margin": float(trace["rel_gap"].min()),
            "min_margin_over_perturbation": float(guard.min())}


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
