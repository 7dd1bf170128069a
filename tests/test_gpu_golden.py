"""GPU parity of the product surfaces against the reference's golden fixtures (tests/golden/).

* G1: VQARetrieval.retrieve_closest_qa_pairs (all return modes, both phases, k in {1,3,5,15},
  exact ties) — ids/prompts/answers/info bit-exact, dists rel 2e-5.
* G2: T5VisionModel.prepare_input / predict / forward + VQARetrieval end to end at reduced size
  — prompts and token ids exact, embeddings FP_TOL, loss 1e-4 abs.
* G3: DeviceT5 at full t5-small size — greedy ids exact, logits FP_TOL, loss 1e-4.
* G4: DeviceViT / DeviceCLIPText at full ViT-B/32 size — FP_TOL.
"""
import json
import os
import sys

import numpy as np
import pytest
import torch

from multimodalpromptretrieval_amd import synthetic as syn

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
sys.path.insert(0, GOLD)
import inputs as gi  # noqa: E402

FP_TOL = 2e-4


def _rel(a, b):
    a = torch.as_tensor(a).detach().float().cpu()
    b = torch.as_tensor(b).detach().float().cpu()
    return float((a - b).abs().max() / b.abs().max())


def _check_dists(got, want, q, X):
    """L2 distances via the cdist mm path carry the cancellation error of |q|^2+|x|^2-2q.x:
    compare squared distances within 2e-6 * (|q|^2 + |x|^2) of the row they belong to (exact
    self-matches are pure rounding noise, ~sqrt(ulp(|x|^2)), in the reference too)."""
    from oracle import retrieval as oret
    got, want = np.asarray(got, np.float64), np.asarray(want, np.float64)
    ids = oret.topk_ids(oret.cdist(q, X), got.shape[1], False).numpy()
    scale = (q.double() ** 2).sum(1).numpy()[:, None] + (X.double() ** 2).sum(1).numpy()[ids]
    assert np.all(np.abs(got ** 2 - want ** 2) <= 2e-6 * scale + 1e-12)


@pytest.fixture(scope="module")
def tiny_retrieval(device):
    from multimodalpromptretrieval_amd.dataset import VQARetrieval
    ccfg, clip_sd, *_ = gi.g2_models()
    return VQARetrieval(device, clip_state_dict=clip_sd, clip_tokenizer=syn.hash_clip_tokenize)


def _with_queries(r, q):
    r.encode_queries = lambda batch: q.to(r.device)   # stub encoder, as the golden generator
    return {"image": torch.zeros(q.shape[0], 1), "question": [f"x{i}" for i in range(q.shape[0])]}


def test_g1_retrieval_product(device, tiny_retrieval):
    with open(os.path.join(GOLD, "g1_retrieval.json")) as f:
        g1 = json.load(f)
    r = tiny_retrieval
    built = {}
    for case in g1["cases"]:
        N, D, k, tr = case["N"], case["D"], case["k"], case["training"]
        if (N, D) not in built:
            X, q, _ = gi.g1_queries(N, D, case["seed"])
            built[(N, D)] = (X, q)
        X, q = built[(N, D)]
        r.set_index(X, syn.answers(N, gi.G1_ANS_VOCAB), gi.question_info(N), k, tr)
        batch = _with_queries(r, q)
        assert r.retrieve_closest_qa_pairs(batch, return_info=["question_id"]) == \
            [[str(i) for i in row] for row in case["ids"]]
        assert r.retrieve_closest_qa_pairs(batch) == case["prompts"]
        assert r.retrieve_closest_qa_pairs(batch, use_quantifier=False) == case["prompts_noq"]
        assert r.retrieve_closest_qa_pairs(batch, return_ans=True) == case["answers"]
        assert r.retrieve_closest_qa_pairs(
            batch, return_info=["question_id", "question_type"]) == case["info"]
        dd = r.retrieve_closest_qa_pairs(batch, return_dists=True)
        assert [a for a, _ in dd] == case["dists_answers"]
        _check_dists(np.stack([d for _, d in dd]), case["dists"], q, X)
    Xt, qt = gi.tie_index()
    for c in g1["ties"]["cases"]:
        r.set_index(Xt, syn.answers(300, 5), gi.question_info(300), c["k"], c["training"])
        batch = _with_queries(r, qt)
        assert r.retrieve_closest_qa_pairs(batch, return_info=["question_id"]) == \
            [[str(i) for i in row] for row in c["ids"]]
        assert r.retrieve_closest_qa_pairs(batch) == c["prompts"]


def test_g2_pipeline_product(device):
    from multimodalpromptretrieval_amd.dataset import VQARetrieval
    from multimodalpromptretrieval_amd.model import T5VisionModel
    z = np.load(os.path.join(GOLD, "g2_pipeline.npz"))
    with open(os.path.join(GOLD, "g2_pipeline.json")) as f:
        j = json.load(f)
    ccfg, clip_sd, tcfg, tok_sd, t5cfg, t5_sd = gi.g2_models()
    X, answers, info = gi.g2_index(ccfg)
    retr = VQARetrieval(device, clip_state_dict=clip_sd, clip_tokenizer=syn.hash_clip_tokenize)
    retr.set_index(X, answers, info, gi.G2["k"], False)
    model = T5VisionModel(device, clip_state_dict=tok_sd, t5_state_dict=t5_sd,
                          tokenizer=syn.HashT5Tokenizer(),
                          retrieval_function=retr.retrieve_closest_qa_pairs)
    model.eval()
    batch = gi.g2_batch()
    q = retr.encode_queries(batch)
    assert _rel(q, z["query"]) < FP_TOL
    assert retr.retrieve_closest_qa_pairs(batch) == j["prompts"]
    combined, mask, enc = model.prepare_input(batch)
    assert enc["input_ids"].tolist() == z["input_ids"].tolist()
    assert mask.cpu().tolist() == z["mask"].tolist()
    assert _rel(combined, z["combined"]) < FP_TOL
    assert model.predict(batch) == j["predictions"]
    assert abs(float(model(batch)) - float(z["loss"])) < 1e-4
    assert retr.retrieve_closest_qa_pairs(batch, use_quantifier=False) == j["prompts_noq"]
    model.use_quantifier = False
    c2, _, e2 = model.prepare_input(batch)
    assert e2["input_ids"].tolist() == z["input_ids_noq"].tolist()
    assert _rel(c2, z["combined_noq"]) < FP_TOL
    model.use_quantifier = True
    model.use_image_info = False
    c3, m3, _ = model.prepare_input(batch)
    assert _rel(c3, z["combined_txt"]) < FP_TOL
    assert m3.cpu().tolist() == z["mask_txt"].tolist()


def test_g2_predict_many_matches_predict(device):
    """The serving pipeline (1-3 generate calls in flight, batch pairs sharing a decode loop or
    not) returns, per batch, exactly predict()'s answers (batches of different prompt lengths
    and images in flight together; the first is the golden one)."""
    from multimodalpromptretrieval_amd.dataset import VQARetrieval
    from multimodalpromptretrieval_amd.model import T5VisionModel
    with open(os.path.join(GOLD, "g2_pipeline.json")) as f:
        j = json.load(f)
    ccfg, clip_sd, tcfg, tok_sd, t5cfg, t5_sd = gi.g2_models()
    X, answers, info = gi.g2_index(ccfg)
    retr = VQARetrieval(device, clip_state_dict=clip_sd, clip_tokenizer=syn.hash_clip_tokenize)
    retr.set_index(X, answers, info, gi.G2["k"], False)
    model = T5VisionModel(device, clip_state_dict=tok_sd, t5_state_dict=t5_sd,
                          tokenizer=syn.HashT5Tokenizer(),
                          retrieval_function=retr.retrieve_closest_qa_pairs).eval()
    b0 = gi.g2_batch()
    batches = [b0]
    for i in (1, 2, 3):
        b = dict(b0)
        b["image"] = syn.images(900 + i, len(b0["question"]), gi.G2["clip_cfg"]["image_size"])
        b["question"] = [q + " which" * (i * k % 5) for k, q in enumerate(b0["question"])]
        batches.append(b)
    want = [model.predict(b) for b in batches]
    want_ans = [retr.retrieve_closest_qa_pairs(b, return_ans=True) for b in batches]
    assert want[0] == j["predictions"]
    assert list(model.predict_many(batches)) == want
    for depth in (1, 3):  # decodes in flight on separate workspace slots
        assert list(model.predict_many(batches, depth)) == want
        assert list(model.predict_many(batches, depth, pair_decodes=False)) == want
        assert list(model.predict_many(batches, depth, lookahead=False)) == want
        assert list(model.predict_many(batches, depth, tower_slots=2)) == want
        assert list(model.predict_many(batches, depth, tower_batches=1)) == want
    assert list(model.predict_many(batches[:3])) == want[:3]  # an unpaired last batch
    for group in (3, 4):  # 3 / 4 batches per decode loop (a partial last group at 3)
        assert list(model.predict_many(batches, decode_group=group)) == want
    assert list(model.predict_many(iter(batches[:1]))) == want[:1]
    assert list(model.predict_many([])) == []
    # main.py-shaped loop with lookahead hints (serving.lookahead): the next batch's towers and
    # scan run beside this batch's decode; every answer and the four analytics calls unchanged
    from multimodalpromptretrieval_amd.serving import lookahead
    for _ in range(2):
        got = []
        for b in lookahead(batches, model):
            assert b is batches[len(got)]
            got.append(model.predict(b))
            assert retr.retrieve_closest_qa_pairs(b, return_ans=True) == want_ans[len(got) - 1]
        assert got == want
    assert not model._hints  # every hint consumed
    # main.py-shaped loop through serving.pipelined (the dropin launcher's default): a serving
    # loop runs ahead, predict() returns its answers, the analytics reuse each batch's search
    from multimodalpromptretrieval_amd.serving import ServingOptions, pipelined
    for slots in (1, 2):
        got = []
        opts = ServingOptions.resolve(tower_slots=slots)
        for b in pipelined(batches, model, opts):
            assert b is batches[len(got)]
            got.append(model.predict(b))
            assert retr.retrieve_closest_qa_pairs(b, return_ans=True) == want_ans[len(got) - 1]
        assert got == want
    model.hint_next(batches[2])  # a hinted batch predicted out of order, another never
    assert model.predict(batches[1]) == want[1] and model.predict(batches[2]) == want[2]
    # training mode (main.py:170-178 under the dropin launcher's lookahead): a hinted batch's
    # forward inputs are the unhinted ones
    model.train()
    assert model.hint_next(batches[0]) is True
    pre = model._take_hint(batches[0])
    with torch.no_grad():
        hinted = model.prepare_input(batches[0], _pre=pre)
        plain = model.prepare_input(batches[0])
    assert torch.equal(hinted[0], plain[0]) and torch.equal(hinted[1], plain[1])
    model.eval()


def test_g2_state_dict_roundtrip_refreshes_device_weights(device):
    from multimodalpromptretrieval_amd.model import T5VisionModel
    _, _, tcfg, tok_sd, t5cfg, t5_sd = gi.g2_models()
    m = T5VisionModel(device, clip_state_dict=tok_sd, t5_state_dict=t5_sd,
                      tokenizer=syn.HashT5Tokenizer())
    batch = gi.g2_batch()
    a, _, _ = m.prepare_input(batch)
    sd = m.state_dict()
    assert "T5_model.shared.weight" in sd and "T5_model.lm_head.weight" in sd
    assert "vision_model.visual.conv1.weight" in sd
    sd2 = {k: (v * 2 if k == "vision_model.visual.proj" else v) for k, v in sd.items()}
    m.load_state_dict(sd2)
    b, _, _ = m.prepare_input(batch)
    assert _rel(b[:, :5], 2 * a[:, :5]) < 1e-5     # image tokens scale with the new proj


@pytest.mark.slow
def test_g3_t5_small_product(device):
    from multimodalpromptretrieval_amd.t5 import DeviceT5
    z = np.load(os.path.join(GOLD, "g3_t5_small.npz"))
    cfg = syn.T5Config()
    sd = syn.t5_state_dict(gi.G3["t5_seed"], cfg)
    m = DeviceT5(sd, device)
    ids, img_tok, mask = gi.g3_inputs(cfg.d_model)
    emb = torch.cat([img_tok, sd["shared.weight"][ids]], 1)
    enc = m.encode(emb, mask)
    assert _rel(enc[:, :8], z["enc_head"]) < FP_TOL
    seqs = m.generate(emb, mask, 20)
    assert seqs.tolist() == z["sequences"].tolist()
    labels = torch.from_numpy(z["labels"])
    dec_in = torch.zeros_like(labels)
    dec_in[:, 1:] = labels[:, :-1]
    dec_in[dec_in == -100] = 0
    lg = m.logits(emb, mask, dec_in)
    assert _rel(lg[:, :, torch.from_numpy(z["vocab_sel"])], z["logits_sel"]) < FP_TOL
    assert lg.argmax(-1).cpu().tolist() == z["logits_argmax"].tolist()
    assert abs(float(m.loss(lg, labels)) - float(z["loss"])) < 1e-4


@pytest.mark.slow
def test_g4_clip_product(device):
    from multimodalpromptretrieval_amd.encoders import CLS, TOKENS, DeviceCLIPText, DeviceViT
    z = np.load(os.path.join(GOLD, "g4_clip_vit_b32.npz"))
    sd = syn.clip_state_dict(gi.G4["clip_seed"])
    img = syn.images(gi.G4["img_seed"], gi.G4["B_img"]).to(device)
    toks = syn.clip_tokens(gi.G4["tok_seed"], gi.G4["B_txt"])
    vit = DeviceViT(sd, device)
    txt = DeviceCLIPText(sd, device)
    assert _rel(vit(img, CLS), z["image_cls"]) < FP_TOL
    assert _rel(vit(img, TOKENS), z["image_tokens"]) < FP_TOL
    assert _rel(txt(toks), z["text"]) < FP_TOL
