"""GPU parity of the configs and surfaces round 1 left unexercised (BASELINE.json configs C1, C5;
SURVEY.md §8 a8), against golden fixtures the reference itself produced (tests/golden/):

* G5 — utils.cosine_similarity (utils.py:57-62): the aligned-row kernel and the
  [B,1,D] x [1,N,D] retrieval-matrix form, values within 2e-6 (cosines are <= 1 in magnitude);
* G6 — config C1, retrieval off (retrieval_function=None, architectures/T5VisionModel.py:148-149):
  token ids / mask exact, embeddings FP_TOL, answers exact, loss 1e-4;
* G7 — config C5's model: t5-base (768 / 12 heads / 3072 / 12+12 layers) behind T5VisionModel with
  use_image_info=0, through predict() / forward() and DeviceT5 directly;
* G8 — a 562-key source (50 image tokens + max_source_length=512 text tokens): the >256-key
  prefill attention and the multi-pass decode cross-attention;
* config C5's scan at full size: 1,048,576 x 512 index, 256 queries, k = 5, ids against an fp64
  host oracle (bit-exact wherever the fp64 distance margin exceeds the fp32 error bound).
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


def test_g5_cosine_similarity_product(device):
    from multimodalpromptretrieval_amd.utils import cosine_similarity
    z = np.load(os.path.join(GOLD, "g5_cosine.npz"))
    for name, x1, x2, dim in gi.g5_inputs():
        # operands produced on a side stream: the drop-in must order itself behind it
        side = torch.cuda.Stream(device)
        with torch.cuda.stream(side):
            a = x1.to(device, non_blocking=True) * 1.0
            b = x2.to(device, non_blocking=True) * 1.0
        torch.cuda.current_stream(device).wait_stream(side)
        got = cosine_similarity(a, b, dim=dim)
        assert tuple(got.shape) == z[name].shape, name
        assert np.abs(got.cpu().numpy() - z[name]).max() <= 2e-6, name


def _g2_parts(device):
    from multimodalpromptretrieval_amd.dataset import VQARetrieval
    ccfg, clip_sd, tcfg, tok_sd, t5cfg, t5_sd = gi.g2_models()
    X, answers, info = gi.g2_index(ccfg)
    retr = VQARetrieval(device, clip_state_dict=clip_sd, clip_tokenizer=syn.hash_clip_tokenize)
    retr.set_index(X, answers, info, gi.G2["k"], False)
    return retr, tok_sd, t5_sd


def test_g6_retrieval_off_product(device):
    """Config C1: predict / forward with no retrieval function."""
    from multimodalpromptretrieval_amd.model import T5VisionModel
    z = np.load(os.path.join(GOLD, "g6_noretrieval.npz"))
    with open(os.path.join(GOLD, "g6_noretrieval.json")) as f:
        j = json.load(f)
    _, tok_sd, t5_sd = _g2_parts(device)
    model = T5VisionModel(device, clip_state_dict=tok_sd, t5_state_dict=t5_sd,
                          tokenizer=syn.HashT5Tokenizer(), retrieval_function=None).eval()
    batch = gi.g2_batch()
    combined, mask, enc = model.prepare_input(batch)
    assert enc["input_ids"].tolist() == z["input_ids"].tolist()
    assert mask.cpu().tolist() == z["mask"].tolist()
    assert _rel(combined, z["combined"]) < FP_TOL
    assert model.predict(batch) == j["predictions"]
    assert abs(float(model(batch)) - float(z["loss"])) < 1e-4
    assert list(model.predict_many([batch, batch])) == [j["predictions"]] * 2


@pytest.mark.slow
def test_g7_t5_base_product(device):
    """Config C5's model: t5-base, use_image_info=0, G2 retrieval prompts."""
    from multimodalpromptretrieval_amd.model import T5VisionModel
    from multimodalpromptretrieval_amd.t5 import DeviceT5
    z = np.load(os.path.join(GOLD, "g7_t5_base.npz"))
    with open(os.path.join(GOLD, "g7_t5_base.json")) as f:
        j = json.load(f)
    retr, tok_sd, _ = _g2_parts(device)
    cfg = syn.T5_BASE
    sd = syn.t5_state_dict(gi.G7["t5_seed"], cfg)
    model = T5VisionModel(device, T5_version="t5-base", use_image_info=False,
                          clip_state_dict=tok_sd, t5_state_dict=sd,
                          tokenizer=syn.HashT5Tokenizer(),
                          retrieval_function=retr.retrieve_closest_qa_pairs).eval()
    batch = gi.g2_batch()
    combined, mask, enc = model.prepare_input(batch)
    assert enc["input_ids"].tolist() == z["input_ids"].tolist()
    assert mask.cpu().tolist() == z["mask"].tolist()
    assert _rel(combined, z["combined"]) < FP_TOL
    assert model.predict(batch) == j["predictions"]
    assert abs(float(model(batch)) - float(z["loss"])) < 1e-4
    m = DeviceT5(sd, device)
    emb = torch.from_numpy(z["combined"])
    msk = torch.from_numpy(z["mask"])
    assert _rel(m.encode(emb, msk)[:, :8], z["enc_head"]) < FP_TOL
    assert m.generate(emb, msk, 20).tolist() == z["sequences"].tolist()
    labels = torch.from_numpy(z["labels"])
    dec_in = torch.zeros_like(labels)
    dec_in[:, 1:] = labels[:, :-1]
    dec_in[dec_in == -100] = 0
    lg = m.logits(emb, msk, dec_in)
    assert _rel(lg[:, :, torch.from_numpy(z["vocab_sel"])], z["logits_sel"]) < FP_TOL
    assert lg.argmax(-1).cpu().tolist() == z["logits_argmax"].tolist()


@pytest.mark.slow
def test_g8_long_source_product(device):
    """L = 562 keys: encoder attention past 256 keys, decode cross-attention in several passes."""
    from multimodalpromptretrieval_amd.t5 import DeviceT5
    z = np.load(os.path.join(GOLD, "g8_long_source.npz"))
    cfg = syn.T5Config()
    sd = syn.t5_state_dict(gi.G8["t5_seed"], cfg)
    m = DeviceT5(sd, device)
    ids, img_tok, mask = gi.g8_inputs(cfg.d_model)
    emb = torch.cat([img_tok, sd["shared.weight"][ids]], 1)
    assert emb.shape[1] == 562
    assert _rel(m.encode(emb, mask)[:, ::37], z["enc_rows"]) < FP_TOL
    assert m.generate(emb, mask, 20).tolist() == z["sequences"].tolist()
    # the long row alone and grouped with a short batch in one decode loop: same tokens
    short_emb, short_mask = emb[1:, :120].contiguous(), mask[1:, :120].contiguous()
    a, b = m.generate_batches_padded([(emb[:1], mask[:1]), (short_emb, short_mask)], 20)
    assert DeviceT5.trim(a).tolist() == z["sequences"][:1, :DeviceT5.trim(a).shape[1]].tolist()
    assert b.tolist() == m.generate_padded(short_emb, short_mask, 20).tolist()
    labels = torch.from_numpy(z["labels"])
    dec_in = torch.zeros_like(labels)
    dec_in[:, 1:] = labels[:, :-1]
    dec_in[dec_in == -100] = 0
    lg = m.logits(emb, mask, dec_in)
    assert _rel(lg[:, :, torch.from_numpy(z["vocab_sel"])], z["logits_sel"]) < FP_TOL
    assert abs(float(m.loss(lg, labels)) - float(z["loss"])) < 1e-4


def _fp64_topk(X, q, k, chunk=1 << 17):
    """fp64 ascending squared-distance top-(k+1) ids and values (random fp32 data has no exact
    fp64 ties, so the order is unambiguous)."""
    qd = q.double()
    qn = (qd * qd).sum(1, keepdim=True)
    best_d = torch.empty((q.shape[0], 0), dtype=torch.float64)
    best_i = torch.empty((q.shape[0], 0), dtype=torch.int64)
    for lo in range(0, X.shape[0], chunk):
        xd = X[lo:lo + chunk].double()
        dd = qn + (xd * xd).sum(1)[None, :] - 2.0 * qd @ xd.T
        v, i = torch.topk(dd, k + 1, dim=1, largest=False, sorted=True)
        best_d, best_i = torch.cat([best_d, v], 1), torch.cat([best_i, i + lo], 1)
        v, o = torch.topk(best_d, k + 1, dim=1, largest=False, sorted=True)
        best_d, best_i = v, torch.gather(best_i, 1, o)
    return best_d, best_i


@pytest.mark.slow
def test_c5_scan_full_size_vs_fp64_oracle(device):
    """Config C5's retrieval core at full size (the bench's c5_scan inputs): every query's k ids
    equal the fp64 ranking wherever neighbouring fp64 distances differ by more than the fp32
    evaluation bound of |q|^2 + |x|^2 - 2 q.x (4e-6 relative to |q|^2 + |x|^2)."""
    from multimodalpromptretrieval_amd.index import DeviceIndex
    n, d, B, k = 1 << 20, 512, 256, 5
    rows = syn.index_rows_device(7, 0, n, d, device)
    g = torch.Generator(device=device).manual_seed(8)
    q = torch.randn((B, d), device=device, generator=g) * 0.3
    ix = DeviceIndex(rows, device)
    dist, ids = ix.search(q, k)
    ids = ids.cpu()
    Xh, qh = rows.cpu(), q.cpu()
    del ix, rows
    torch.cuda.empty_cache()
    best_d, best_i = _fp64_topk(Xh, qh, k)
    scale = (qh.double() ** 2).sum(1, keepdim=True) + (Xh.double() ** 2).sum(1)[best_i]
    tol = 4e-6 * scale
    gap = (best_d[:, 1:] - best_d[:, :-1]) > tol[:, 1:]     # rank r and r+1 are separable
    exact = (ids == best_i[:, :k])
    n_exact = int(exact.all(1).sum())
    for r in range(B):
        for c in range(k):
            # position c is pinned when it is separated from both neighbours in the fp64 order
            pinned = (c == 0 or bool(gap[r, c - 1])) and bool(gap[r, c])
            if pinned:
                assert int(ids[r, c]) == int(best_i[r, c]), (r, c, ids[r], best_i[r])
    gd = (qh.double()[:, None, :] - Xh.double()[ids]).pow(2).sum(-1)
    assert torch.all(gd[:, -1] <= best_d[:, k - 1] + tol[:, k - 1])
    print(f"C5 scan: {n_exact}/{B} queries bit-exact in all {k} ids")
    assert n_exact >= B - 2


@pytest.mark.parametrize("n,d,b,k", [(50000, 512, 128, 5), (20011, 256, 64, 8), (3000, 512, 300, 1),
                                     (30001, 256, 200, 3), (131072, 512, 256, 5)])
def test_coarse_scan_matches_oracle(device, n, d, b, k):
    """Large-batch L2 searches take the bf16 coarse scan + exact fp32 re-rank: ids equal the
    exact ranking wherever fp64 separates neighbours by more than the fp32 bound."""
    from multimodalpromptretrieval_amd.index import DeviceIndex
    X = syn.index_rows(1000 + n, n, d)
    q = syn.index_rows(2000 + n, b, d)
    q[:4] = X[[5, 17, n - 1, n // 2]]                      # exact self matches included
    dist, ids = DeviceIndex(X, device).search(q, k)
    ids = ids.cpu()
    best_d, best_i = _fp64_topk(X, q, k)
    scale = (q.double() ** 2).sum(1, keepdim=True) + (X.double() ** 2).sum(1)[best_i]
    gap = (best_d[:, 1:] - best_d[:, :-1]) > 4e-6 * scale[:, 1:]
    for r in range(b):
        for c in range(k):
            if (c == 0 or bool(gap[r, c - 1])) and bool(gap[r, c]):
                assert int(ids[r, c]) == int(best_i[r, c]), (r, c)
    # squared distances within the cdist mm-path cancellation bound (exact self matches are
    # rounding noise, ~sqrt(ulp(|x|^2)), in the reference too)
    got2 = dist.cpu().double() ** 2
    assert torch.all((got2 - best_d[:, :k]).abs() <= 2e-6 * scale[:, :k] + 1e-9)


def test_coarse_scan_falls_back_on_a_dense_neighbourhood(device):
    """Forty rows within the coarse error bound of query 0 overflow its coarse candidates: the
    query's device flag runs the exact scan for it, and its ids are still the exact ones (lowest
    id on the exact tie the duplicated row creates)."""
    from multimodalpromptretrieval_amd.index import DeviceIndex
    n, d, b, k = 20000, 512, 64, 5
    X = syn.index_rows(31, n, d)
    q = syn.index_rows(32, b, d)
    base = q[0] + 0.05
    noise = syn.index_rows(33, 40, d) * 1e-4
    X[1000:1040] = base + noise
    X[7000] = X[1003]                   # an exact duplicate: tie -> lowest id first
    ix = DeviceIndex(X, device)
    dist, ids = ix.search(q, k)
    assert ix.coarse_fallbacks() >= 1
    ids = ids.cpu()
    best_d, best_i = _fp64_topk(X, q, k)
    scale = (q.double() ** 2).sum(1, keepdim=True) + (X.double() ** 2).sum(1)[best_i]
    gap = (best_d[:, 1:] - best_d[:, :-1]) > 4e-6 * scale[:, 1:]
    for r in range(b):
        for c in range(k):
            if (c == 0 or bool(gap[r, c - 1])) and bool(gap[r, c]):
                assert int(ids[r, c]) == int(best_i[r, c]), (r, c)
    row0 = ids[0].tolist()
    assert all(1000 <= j < 1040 or j == 7000 for j in row0)
    if 7000 in row0:
        assert 1003 in row0 and row0.index(1003) < row0.index(7000)
    # a batch with no dense neighbourhood takes (almost) no fallback
    ix2 = DeviceIndex(syn.index_rows(34, n, d), device)
    ix2.search(q, k)
    assert 0 <= ix2.coarse_fallbacks() <= 1


@pytest.mark.parametrize("k", [1, 3])
def test_c2_full_size_end_to_end_vs_oracle(device, k):
    """Config C2 (C3's k = 3 too) end to end at full size: a 6,500 x 1,024 index, two seeded
    ViT-B/32 towers + CLIP text, t5-small, batches of 16 with real-algorithm tokenizers and host
    images — T5VisionModel.predict() and the retrieval prompts on the device against
    oracle/pipeline.py (torch-CPU fp32 restatement of the reference path, the CPU baseline's
    code) on the same weights and batches: retrieved prompts and greedy answers equal."""
    from multimodalpromptretrieval_amd.dataset import VQARetrieval
    from multimodalpromptretrieval_amd.model import T5VisionModel
    from multimodalpromptretrieval_amd.tokenization import SpmT5Tokenizer, clip_tokenize
    from oracle import pipeline
    N, D, B = 6500, 1024, 16
    retr_sd, tok_sd, t5_sd = syn.clip_state_dict(1), syn.clip_state_dict(2), syn.t5_state_dict(3)
    X = syn.index_rows(4, N, D)
    answers = syn.answers(N, 50)
    info = {"question_id": [str(j) for j in range(N)], "question_type": ["open"] * N,
            "question": [""] * N}
    retr = VQARetrieval(device, clip_state_dict=retr_sd, clip_tokenizer=clip_tokenize)
    retr.set_index(X, answers, info, k, is_training_phase=False)
    model = T5VisionModel(device, clip_state_dict=tok_sd, t5_state_dict=t5_sd,
                          tokenizer=SpmT5Tokenizer(),
                          retrieval_function=retr.retrieve_closest_qa_pairs).eval()
    rng = np.random.Generator(np.random.PCG64(77))
    words = ["what", "is", "the", "organ", "shown", "in", "this", "image", "lung", "left",
             "abnormal", "scan", "where", "does", "it", "appear", "brain", "chest", "liver"]
    ref_tok = SpmT5Tokenizer()
    ref_tok.add_tokens(["[itk]"])
    for bi in range(2):
        batch = {"image": syn.images(900 + bi, B),
                 "question": [" ".join(rng.choice(words, size=int(rng.integers(5, 14)))) + "?"
                              for _ in range(B)],
                 "task": ["vqa"] * B, "answer": ["yes"] * B,
                 "question_id": [str(bi * B + j) for j in range(B)],
                 "question_type": ["open"] * B}
        with torch.no_grad():
            got = model.predict(batch)
            got_prompts = retr.retrieve_closest_qa_pairs(batch)
            preds, prompts, _ = pipeline.predict(
                batch, retr_sd, tok_sd, t5_sd, 8, X, answers, info, k, False, clip_tokenize,
                ref_tok, 20, forced_steps=True)
        assert got_prompts == prompts, f"batch {bi}: retrieved prompts differ"
        assert got == preds, f"batch {bi}: greedy answers differ"
