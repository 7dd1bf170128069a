"""Oracle: the whole predict() path on the CPU (TEST INFRASTRUCTURE ONLY; also the timed
CPU baseline of bench.py).

Restates architectures/T5VisionModel.py:141-216 (prepare_input + predict) with the retrieval
function of dataset/VQAFeatureDataset.py:187-246, in torch-CPU fp32 eager ops.
"""
from __future__ import annotations

import torch

from . import clip as oclip
from . import retrieval as oret
from . import t5 as ot5


def predict(batch: dict, retrieval_clip_sd: dict, token_clip_sd: dict, t5_sd: dict,
            t5_heads: int, index: torch.Tensor, answers: list, question_info: dict, k: int,
            is_training_phase: bool, clip_tokenize, t5_tokenizer, max_new_tokens: int = 20,
            forced_steps: bool = False, use_quantifier: bool = True, trace: dict = None):
    """Returns (answers, prompts, tokens).  With ``trace`` (a dict) the retrieval's details are
    also recorded there: ``query`` [B, D] fp32, ``ids`` [B, k] int64 (the rows the prompts were
    built from, dataset/VQAFeatureDataset.py:194-197), ``dists`` [B, k] fp32 (the
    ``return_dists`` values, :242-245) and the fp64 rank margins of ``retrieval.rank_margins``
    (``gap``, ``rel_gap``, ``d_last``)."""
    img = batch["image"].float().cpu()
    if k > 0:
        q = torch.cat([oclip.encode_image(retrieval_clip_sd, img),
                       oclip.encode_text(retrieval_clip_sd, clip_tokenize(batch["question"]))], 1)
        prompts = oret.retrieve_closest_qa_pairs(q, index, answers, question_info, k,
                                                 is_training_phase,
                                                 use_quantifier=use_quantifier)
        if trace is not None:
            trace["query"] = q
            trace["ids"] = oret.topk_ids(oret.cdist(q, index), k, is_training_phase)
            trace["dists"] = oret.smallest_dists(q, index, k)
            trace["gap"], trace["rel_gap"], trace["d_last"] = oret.rank_margins(
                q, index, k, is_training_phase)
    else:
        prompts = ["" for _ in batch["task"]]                 # retrieval off
    img_tok = oclip.image_token_features(token_clip_sd, img)
    sents = [f"Answer the {t} question: " + qq + p
             for t, qq, p in zip(batch["task"], batch["question"], prompts)]
    enc = t5_tokenizer(sents, padding="longest", max_length=512, truncation=True,
                       return_tensors="pt")
    emb = torch.cat([img_tok, t5_sd["shared.weight"][enc["input_ids"]]], 1)
    mask = torch.cat([torch.ones(img_tok.shape[:2]), enc["attention_mask"].float()], 1)
    toks = ot5.generate_cached(t5_sd, emb, mask, t5_heads, max_new_tokens,
                               forced_steps=forced_steps)
    return t5_tokenizer.batch_decode(toks, skip_special_tokens=True), prompts, toks
