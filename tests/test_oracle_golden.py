"""Pin the CPU oracle against the golden fixtures captured from the reference (CPU only).

G1: dataset/VQAFeatureDataset.py:187-246 run by the reference itself (ids, prompts, answers,
    info, dists, both phases, k in {1,3,5,15}, exact-tie cases).
G2: architectures/T5VisionModel.py:141-234 run by the reference itself at reduced size.
G3/G4: transformers T5 / CLIP (the third-party arithmetic's second source) at full size.
"""
import json
import os
import sys

import numpy as np
import pytest
import torch

from multimodalpromptretrieval_amd import synthetic as syn
from oracle import clip as oclip
from oracle import retrieval as oret
from oracle import t5 as ot5

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
sys.path.insert(0, GOLD)
import inputs as gi  # noqa: E402

FP_TOL = 1e-4


def _g1():
    with open(os.path.join(GOLD, "g1_retrieval.json")) as f:
        return json.load(f)


def _rel(a, b):
    a = torch.as_tensor(a).float()
    b = torch.as_tensor(b).float()
    return float((a - b).abs().max() / b.abs().max())


@pytest.mark.parametrize("case_idx", range(16))
def test_g1_retrieval_oracle(case_idx):
    case = _g1()["cases"][case_idx]
    N, D, k, tr = case["N"], case["D"], case["k"], case["training"]
    X, q, _ = gi.g1_queries(N, D, case["seed"])
    answers = syn.answers(N, gi.G1_ANS_VOCAB)
    info = gi.question_info(N)
    ids = oret.topk_ids(oret.cdist(q, X), k, tr)
    assert ids.tolist() == case["ids"]
    assert oret.retrieve_closest_qa_pairs(q, X, answers, info, k, tr) == case["prompts"]
    assert oret.retrieve_closest_qa_pairs(q, X, answers, info, k, tr,
                                          use_quantifier=False) == case["prompts_noq"]
    assert oret.retrieve_closest_qa_pairs(q, X, answers, info, k, tr,
                                          return_ans=True) == case["answers"]
    assert oret.retrieve_closest_qa_pairs(
        q, X, answers, info, k, tr, return_info=["question_id", "question_type"]) == case["info"]
    dd = oret.retrieve_closest_qa_pairs(q, X, answers, info, k, tr, return_dists=True)
    assert [a for a, _ in dd] == case["dists_answers"]
    np.testing.assert_allclose(np.stack([d for _, d in dd]), np.array(case["dists"]),
                               rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("case_idx", [0, 5, 11])
def test_id_parity_checker_on_g1(case_idx):
    """The full-size id checker (oracle.retrieval.id_parity): the G1 ids / dists the reference
    returned pass it against the oracle's trace; a swapped id, a perturbed distance fail; the
    rank margins are the fp64 gaps at rank k / k+1."""
    case = _g1()["cases"][case_idx]
    N, D, k, tr = case["N"], case["D"], case["k"], case["training"]
    X, q, _ = gi.g1_queries(N, D, case["seed"])
    trace = {"query": q, "ids": oret.topk_ids(oret.cdist(q, X), k, tr),
             "dists": oret.smallest_dists(q, X, k)}
    trace["gap"], trace["rel_gap"], trace["d_last"] = oret.rank_margins(q, X, k, tr)
    par = oret.id_parity(case["ids"], case["dists"], q, trace)
    assert par["ids_equal"] and par["dists_within_bound"]
    assert par["max_query_delta"] == 0.0
    assert (trace["gap"] >= 0).all()
    d2 = ((q.double()[:, None, :] - X.double()[None]) ** 2).sum(-1)
    srt = d2.sort(1).values
    s = 1 if tr else 0
    torch.testing.assert_close(trace["gap"], srt[:, s + k] - srt[:, s + k - 1], rtol=1e-9,
                               atol=1e-9)
    bad = [list(r) for r in case["ids"]]
    bad[0][0] = (bad[0][0] + 1) % N
    assert oret.id_parity(bad, case["dists"], q, trace)["ids_equal_rows"] == len(bad) - 1
    far = np.array(case["dists"]) * 1.01
    assert not oret.id_parity(case["ids"], far, q, trace)["dists_within_bound"]


def test_g1_ties_oracle():
    Xt, qt = gi.tie_index()
    ans = syn.answers(300, 5)
    for c in _g1()["ties"]["cases"]:
        ids = oret.topk_ids(oret.cdist(qt, Xt), c["k"], c["training"])
        assert ids.tolist() == c["ids"]
        assert oret.retrieve_closest_qa_pairs(qt, Xt, ans, gi.question_info(300), c["k"],
                                              c["training"]) == c["prompts"]


def test_vote_prompt_buckets():
    # dataset/VQAFeatureDataset.py:222-230: first-inserted answer wins ties; int(certainty*5)
    assert oret.vote_prompt(["a"]) == "I believe the answer is certainly a"
    assert oret.vote_prompt(["a", "b", "c"]) == "I believe the answer is unlikely a"
    assert oret.vote_prompt(["b", "a", "a"]) == "I believe the answer is likely a"
    assert oret.vote_prompt(["b", "a", "a", "b"]) == "I believe the answer is maybe b"
    assert oret.vote_prompt(["x", "y"], False) == "The most frequent answer is x"


def test_cosine_similarity_oracle_matches_reference_golden():
    """G5: the reference's own utils.cosine_similarity (utils.py:57-62) outputs."""
    z = np.load(os.path.join(GOLD, "g5_cosine.npz"))
    for name, x1, x2, dim in gi.g5_inputs():
        got = oret.cosine_similarity(x1, x2, dim=dim)
        assert got.shape == z[name].shape, name
        assert np.abs(got.numpy() - z[name]).max() <= 1e-6, name


def test_g6_retrieval_off_oracle():
    """G6 (config C1): the reference's prepare_input / predict / forward with
    retrieval_function=None (retrieved_info = "", architectures/T5VisionModel.py:148-149)."""
    z = np.load(os.path.join(GOLD, "g6_noretrieval.npz"))
    with open(os.path.join(GOLD, "g6_noretrieval.json")) as f:
        j = json.load(f)
    ccfg, clip_sd, tcfg, tok_sd, t5cfg, t5_sd = gi.g2_models()
    batch = gi.g2_batch()
    tok = syn.HashT5Tokenizer()
    tok.add_tokens(["[itk]"])
    emb, mask, enc = _oracle_prepare(batch, [""] * len(batch["question"]), tok_sd, t5_sd, tok)
    assert enc["input_ids"].tolist() == z["input_ids"].tolist()
    assert mask.tolist() == z["mask"].tolist()
    assert _rel(emb, z["combined"]) < FP_TOL
    seqs, _ = ot5.generate(t5_sd, emb, mask, t5cfg.num_heads, 20)
    assert seqs.tolist() == z["sequences"].tolist()
    assert tok.batch_decode(seqs, skip_special_tokens=True) == j["predictions"]
    from oracle import pipeline
    X, answers, info = gi.g2_index(ccfg)
    preds, prompts, _ = pipeline.predict(
        batch, clip_sd, tok_sd, t5_sd, t5cfg.num_heads, X, answers, info, 0, False,
        syn.hash_clip_tokenize, tok)
    assert prompts == [""] * len(batch["question"]) and preds == j["predictions"]


@pytest.fixture(scope="module")
def g2():
    z = np.load(os.path.join(GOLD, "g2_pipeline.npz"))
    with open(os.path.join(GOLD, "g2_pipeline.json")) as f:
        j = json.load(f)
    return z, j


def _oracle_prepare(batch, prompts, tok_sd, t5_sd, tok):
    img_tok = oclip.image_token_features(tok_sd, batch["image"])
    sents = [f"Answer the {t} question: " + q + p
             for t, q, p in zip(batch["task"], batch["question"], prompts)]
    enc = tok(sents, padding="longest", max_length=512, truncation=True, return_tensors="pt")
    q_emb = t5_sd["shared.weight"][enc["input_ids"]]
    mask = torch.cat([torch.ones(img_tok.shape[:2]), enc["attention_mask"]], 1)
    return torch.cat([img_tok, q_emb], 1), mask, enc


def test_g2_pipeline_oracle(g2):
    z, j = g2
    ccfg, clip_sd, tcfg, tok_sd, t5cfg, t5_sd = gi.g2_models()
    X, answers, info = gi.g2_index(ccfg)
    batch = gi.g2_batch()
    q = torch.cat([oclip.encode_image(clip_sd, batch["image"]),
                   oclip.encode_text(clip_sd, syn.hash_clip_tokenize(batch["question"]))], 1)
    assert _rel(q, z["query"]) < FP_TOL
    prompts = oret.retrieve_closest_qa_pairs(q, X, answers, info, gi.G2["k"], False)
    assert prompts == j["prompts"]
    tok = syn.HashT5Tokenizer()
    tok.add_tokens(["[itk]"])
    emb, mask, enc = _oracle_prepare(batch, prompts, tok_sd, t5_sd, tok)
    assert enc["input_ids"].tolist() == z["input_ids"].tolist()
    assert mask.tolist() == z["mask"].tolist()
    assert _rel(emb, z["combined"]) < FP_TOL
    seqs, _ = ot5.generate(t5_sd, emb, mask, t5cfg.num_heads, 20)
    assert seqs.tolist() == z["sequences"].tolist()
    assert tok.batch_decode(seqs, skip_special_tokens=True) == j["predictions"]
    from oracle import pipeline
    preds, prompts2, _ = pipeline.predict(
        batch, clip_sd, tok_sd, t5_sd, t5cfg.num_heads, X, answers, info, gi.G2["k"], False,
        syn.hash_clip_tokenize, tok)
    assert prompts2 == j["prompts"] and preds == j["predictions"]
    labels = torch.tensor(tok(batch["answer"], padding="longest", max_length=128,
                              truncation=True)["input_ids"])
    labels[labels == 0] = -100
    enc_out = ot5.encode(t5_sd, emb, mask, t5cfg.num_heads)
    logits = ot5.decoder_logits(t5_sd, enc_out, mask, ot5.shift_right(labels), t5cfg.num_heads)
    assert abs(float(ot5.lm_loss(logits, labels)) - float(z["loss"])) < 1e-4


@pytest.mark.slow
def test_g3_t5_small_oracle():
    z = np.load(os.path.join(GOLD, "g3_t5_small.npz"))
    cfg = syn.T5Config()
    sd = syn.t5_state_dict(gi.G3["t5_seed"], cfg)
    ids, img_tok, mask = gi.g3_inputs(cfg.d_model)
    emb = torch.cat([img_tok, sd["shared.weight"][ids]], 1)
    enc = ot5.encode(sd, emb, mask, cfg.num_heads)
    assert _rel(enc[:, :8], z["enc_head"]) < FP_TOL
    seqs, _ = ot5.generate(sd, emb, mask, cfg.num_heads, 20)
    assert seqs.tolist() == z["sequences"].tolist()
    assert ot5.generate_cached(sd, emb, mask, cfg.num_heads, 20).tolist() == seqs.tolist()
    labels = torch.from_numpy(z["labels"])
    lg = ot5.decoder_logits(sd, enc, mask, ot5.shift_right(labels), cfg.num_heads)
    assert _rel(lg[:, :, torch.from_numpy(z["vocab_sel"])], z["logits_sel"]) < FP_TOL
    assert lg.argmax(-1).tolist() == z["logits_argmax"].tolist()
    assert abs(float(ot5.lm_loss(lg, labels)) - float(z["loss"])) < 1e-4


@pytest.mark.slow
def test_g4_clip_oracle():
    z = np.load(os.path.join(GOLD, "g4_clip_vit_b32.npz"))
    sd = syn.clip_state_dict(gi.G4["clip_seed"])
    img = syn.images(gi.G4["img_seed"], gi.G4["B_img"])
    toks = syn.clip_tokens(gi.G4["tok_seed"], gi.G4["B_txt"])
    assert _rel(oclip.encode_image(sd, img), z["image_cls"]) < FP_TOL
    assert _rel(oclip.image_token_features(sd, img), z["image_tokens"]) < FP_TOL
    assert _rel(oclip.encode_text(sd, toks), z["text"]) < FP_TOL


def test_t5_bucket_lut_matches_reference_function():
    from multimodalpromptretrieval_amd.t5 import relative_position_bucket as prod_bucket
    rel = torch.arange(-700, 701)
    for bid in (True, False):
        assert torch.equal(prod_bucket(rel, bid), ot5.relative_position_bucket(rel, bid))


@pytest.mark.slow
def test_g7_t5_base_oracle():
    """G7 (config C5's model): t5-base behind the reference's T5VisionModel, use_image_info=0."""
    z = np.load(os.path.join(GOLD, "g7_t5_base.npz"))
    cfg = syn.T5_BASE
    sd = syn.t5_state_dict(gi.G7["t5_seed"], cfg)
    ids = torch.from_numpy(z["input_ids"])
    mask = torch.from_numpy(z["mask"])
    emb = sd["shared.weight"][ids]
    assert _rel(emb, z["combined"]) < FP_TOL
    enc = ot5.encode(sd, emb, mask, cfg.num_heads)
    assert _rel(enc[:, :8], z["enc_head"]) < FP_TOL
    assert ot5.generate_cached(sd, emb, mask, cfg.num_heads, 20).tolist() == \
        z["sequences"].tolist()
    labels = torch.from_numpy(z["labels"])
    lg = ot5.decoder_logits(sd, enc, mask, ot5.shift_right(labels), cfg.num_heads)
    assert _rel(lg[:, :, torch.from_numpy(z["vocab_sel"])], z["logits_sel"]) < FP_TOL


@pytest.mark.slow
def test_g8_long_source_oracle():
    """G8: a 562-key source (50 image tokens + max_source_length 512 text tokens)."""
    z = np.load(os.path.join(GOLD, "g8_long_source.npz"))
    cfg = syn.T5Config()
    sd = syn.t5_state_dict(gi.G8["t5_seed"], cfg)
    ids, img_tok, mask = gi.g8_inputs(cfg.d_model)
    emb = torch.cat([img_tok, sd["shared.weight"][ids]], 1)
    enc = ot5.encode(sd, emb, mask, cfg.num_heads)
    assert _rel(enc[:, ::37], z["enc_rows"]) < FP_TOL
    assert ot5.generate_cached(sd, emb, mask, cfg.num_heads, 20).tolist() == \
        z["sequences"].tolist()


def test_dropout_oracle_masks():
    """oracle/dropout.py (the device step's counter-based masks): density, scale, determinism,
    independence between sites and seeds."""
    from oracle import dropout as od
    n = 1 << 18
    for p in (0.1, 0.3):
        a = od.factors(5, 3, (n,), p)
        assert abs(float((a != 0).float().mean()) - (1 - p)) < 5e-3
        assert float(a.max()) == float(np.float32(1 / (1 - p))) and float(a.min()) == 0.0
        assert torch.equal(a, od.factors(5, 3, (n,), p))
        b, c = od.factors(5, 4, (n,), p), od.factors(6, 3, (n,), p)
        for o in (b, c):
            agree = float(((a != 0) == (o != 0)).float().mean())
            assert abs(agree - ((1 - p) ** 2 + p ** 2)) < 5e-3  # independent masks
    assert bool((od.factors(1, 1, (64,), 0.0) == 1.0).all())
