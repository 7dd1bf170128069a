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


@pytest.mark.parametrize("s1,s2,dim", [((8, 64), (1, 64), 1),        # [B,D] x [1,D]
                                       ((64,), (10, 64), -1),       # a vector against rows
                                       ((5, 3, 32), (5, 1, 32), 2),
                                       ((7, 40, 3), (1, 40, 3), 1),  # reduce a middle axis
                                       ((6, 33), (6, 33), 0),        # aligned, dim 0
                                       ((4, 1, 16), (1, 9, 16), 2),  # D % 16 != 0 not needed
                                       ((3, 5), (5,), -1),           # fewer dims
                                       ((2, 3, 4), (1, 4), 1),       # positive dim, fewer dims
                                       ((2, 3, 4), (3, 1), -2),
                                       ((2, 1, 5), (3, 1), -1),      # size-1 reduced axis
                                       ((), (), 0)])
def test_cosine_similarity_broadcasting(device, s1, s2, dim):
    """utils.cosine_similarity over the reference's general broadcasting (utils.py:57-62):
    every layout against the oracle restatement of the reference formula in fp64."""
    from multimodalpromptretrieval_amd.utils import cosine_similarity
    from oracle import retrieval as oret
    g = torch.Generator().manual_seed(len(s1) * 10 + len(s2) + dim)
    x1 = torch.randn(s1, generator=g)
    x2 = torch.randn(s2, generator=g)
    if len(s1) == 2 and s1[0] == 8:
        x1[3] = 0  # the eps clamp
    want = oret.cosine_similarity(x1.double(), x2.double(), dim=dim)
    got = cosine_similarity(x1.to(device), x2.to(device), dim=dim)
    assert got.device.type == "cuda" and got.dtype == torch.float32
    assert tuple(got.shape) == tuple(want.shape)
    assert (got.cpu().double() - want).abs().max() <= 2e-6
    # host tensors in, host tensor out (computed on the GPU); the inputs' dtype out
    h = cosine_similarity(x1.half(), x2.half(), dim=dim)
    assert h.device.type == "cpu" and h.dtype == torch.float16
    assert (h.double() - oret.cosine_similarity(x1.half().double(), x2.half().double(),
                                                dim=dim)).abs().max() <= 1e-3


def test_cosine_similarity_errors_as_torch(device):
    from multimodalpromptretrieval_amd.utils import cosine_similarity
    from oracle import retrieval as oret
    with pytest.raises(IndexError):  # the reference too: norm(x2, 2, 1) of a 1-d x2
        oret.cosine_similarity(torch.randn(3, 5), torch.randn(5), dim=1)
    with pytest.raises(IndexError):
        cosine_similarity(torch.randn(3, 5, device=device), torch.randn(5, device=device), dim=1)
    a = torch.randn(4, 8, device=device)
    with pytest.raises(RuntimeError):
        cosine_similarity(a, torch.randn(3, 8, device=device))  # not broadcastable
    with pytest.raises(IndexError):
        cosine_similarity(a, a, dim=2)
    with pytest.raises(RuntimeError):
        cosine_similarity(a, a.cpu())


def _check_topk(ids, vals, ref64, k, descending=False):
    """ids/vals [b, k] against an fp64 score matrix: the selected rows' fp64 scores equal the
    reference's sorted top-k within fp32 rounding (so the set and the order are right up to
    near-ties), every distinct id, and the returned values are those rows' scores."""
    ids = ids.cpu().long()
    order = torch.argsort(-ref64 if descending else ref64, dim=1, stable=True)[:, :k]
    want = torch.gather(ref64, 1, order)
    got = torch.gather(ref64, 1, ids)
    tol = 1e-5 * ref64.abs().max()
    assert (got - want).abs().max() <= tol
    assert all(len(set(r)) == k for r in ids.tolist())
    assert (vals.cpu().double() - got).abs().max() <= tol


@pytest.mark.parametrize("n,d,b,k", [(6500, 1024, 16, 100), (300, 64, 5, 300),
                                     (20000, 512, 3, 4096), (70000, 256, 2, 65)])
def test_scan_large_k(device, n, d, b, k):
    """k > 64 (the reference slices any retrieval_k out of a full argsort,
    dataset/VQAFeatureDataset.py:194-197): the selected rows and their order against fp64 up to
    fp32 near-ties, exact duplicates to the lowest id, both metrics, and the merge of two shards'
    candidates (a sharded search's second stage)."""
    from multimodalpromptretrieval_amd.index import COSINE, DeviceIndex, topk_merge
    X = syn.index_rows(21, n, d)
    X[n // 2] = X[n // 3]  # an exact tie
    q = syn.index_rows(22, b, d)
    q[0] = X[n // 3]
    ref64 = torch.cdist(q.double(), X.double())
    ix = DeviceIndex(X, device)
    dist, ids = ix.search(q.to(device), k)
    _check_topk(ids, dist, ref64, k)
    assert ids[0, :2].cpu().tolist() == [n // 3, n // 2]  # the tie: lowest id first
    Xn, qn = X.double() / X.double().norm(dim=1, keepdim=True), q.double()
    sim64 = (qn / qn.norm(dim=1, keepdim=True)) @ Xn.T
    sim, idc = DeviceIndex(X, device, metric=COSINE).search(q.to(device), k)
    _check_topk(idc, sim, sim64, k, descending=True)
    half = n // 2
    d0, i0 = DeviceIndex(X[:half], device).search(q.to(device), min(k, half))
    d1, i1 = DeviceIndex(X[half:], device, row_offset=half).search(q.to(device), min(k, n - half))
    md, mi = topk_merge(torch.cat([d0, d1], 1), torch.cat([i0, i1], 1), k)
    _check_topk(mi, md, ref64, k)
    assert torch.equal(mi.cpu(), ids.cpu())


def test_retrieval_k_beyond_rows(device):
    """retrieval_k larger than the index (and k = 100): the reference's argsort slice returns
    what there is; answers / prompts / dists as the oracle's."""
    from multimodalpromptretrieval_amd.dataset import VQARetrieval
    from oracle import retrieval as oret
    ccfg, clip_sd, *_ = gi.g2_models()
    for N, k, train in ((40, 100, False), (40, 100, True), (300, 100, False)):
        # well separated distances (|x_j| = 1 + 0.05 j in shuffled order, queries near 0): the
        # order is the same in any precision
        g = torch.Generator().manual_seed(N + k)
        u = torch.randn(N, 2 * ccfg.embed_dim, generator=g)
        scale = 1 + 0.05 * torch.randperm(N, generator=g).float()
        X = u / u.norm(dim=1, keepdim=True) * scale[:, None]
        answers = syn.answers(N, 7)
        info = {"question_id": [str(j) for j in range(N)],
                "question_type": ["open"] * N, "question": [f"q{j}" for j in range(N)]}
        r = VQARetrieval(device, clip_state_dict=clip_sd, clip_tokenizer=syn.hash_clip_tokenize)
        r.set_index(X, answers, info, k, train)
        q = torch.randn(6, 2 * ccfg.embed_dim, generator=g) * 1e-3
        r.encode_queries = lambda batch, q=q: q.to(device)
        batch = {"image": torch.zeros(6, 1), "question": [f"x{i}" for i in range(6)]}
        s = 1 if train else 0
        ids = oret.topk_ids(oret.cdist(q, X), N, skip_first=False)[:, s:s + k]
        want_ans = [[answers[j] for j in row] for row in ids.tolist()]
        assert r.retrieve_closest_qa_pairs(batch, return_ans=True) == want_ans
        dists = r.retrieve_closest_qa_pairs(batch, return_dists=True)
        assert all(len(dd) == min(k, N) for _, dd in dists)


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


@pytest.mark.parametrize("N,k", [(6500, 1), (6500, 3), (10000, 3)])
def test_c2_full_size_end_to_end_vs_oracle(device, N, k):
    """Config C2 (k = 1) and C3 (k = 3 over the combined SLAKE + VQA_RAD index, ~10,000 rows)
    end to end at full size: a 6,500 (10,000) x 1,024 index, two seeded
    ViT-B/32 towers + CLIP text, t5-small, batches of 16 with real-algorithm tokenizers and host
    images — T5VisionModel.predict() and the retrieval prompts on the device against
    oracle/pipeline.py (torch-CPU fp32 restatement of the reference path, the CPU baseline's
    code) on the same weights and batches: the retrieved example ids (``return_info=
    ["question_id"]``, dataset/VQAFeatureDataset.py:202-210) bit-exact, the ``return_dists``
    values within the cdist bound, prompts and greedy answers equal — for predict() and for the
    serving loop (predict_many, the path the headline times).  The fp64 rank-k / rank-k+1
    margin of every query is reported against what the device / CPU query difference can move
    (SURVEY.md §7 hard part (i))."""
    from multimodalpromptretrieval_amd.dataset import VQARetrieval
    from multimodalpromptretrieval_amd.model import T5VisionModel
    from multimodalpromptretrieval_amd.tokenization import SpmT5Tokenizer, clip_tokenize
    from oracle import pipeline
    from oracle import retrieval as oret
    D, B = 1024, 16
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
    batches, want = [], []
    for bi in range(2):
        batch = {"image": syn.images(900 + bi, B),
                 "question": [" ".join(rng.choice(words, size=int(rng.integers(5, 14)))) + "?"
                              for _ in range(B)],
                 "task": ["vqa"] * B, "answer": ["yes"] * B,
                 "question_id": [str(bi * B + j) for j in range(B)],
                 "question_type": ["open"] * B}
        trace = {}
        with torch.no_grad():
            got = model.predict(batch)
            got_prompts = retr.retrieve_closest_qa_pairs(batch)
            got_ids = [[int(s) for s in row]
                       for row in retr.retrieve_closest_qa_pairs(batch, return_info=["question_id"])]
            got_dists = [d for _, d in retr.retrieve_closest_qa_pairs(batch, return_dists=True)]
            q_dev = retr.encode_queries(batch).cpu()
            preds, prompts, _ = pipeline.predict(
                batch, retr_sd, tok_sd, t5_sd, 8, X, answers, info, k, False, clip_tokenize,
                ref_tok, 20, forced_steps=True, trace=trace)
        par = oret.id_parity(got_ids, got_dists, q_dev, trace)
        print(f"batch {bi}: {par}")
        assert par["ids_equal"], f"batch {bi}: retrieved ids differ: {got_ids} vs {trace['ids']}"
        assert par["dists_within_bound"], f"batch {bi}: return_dists outside the bound: {par}"
        assert got_prompts == prompts, f"batch {bi}: retrieved prompts differ"
        assert got == preds, f"batch {bi}: greedy answers differ"
        batches.append(batch)
        want.append(preds)
    # the serving loop (T5VisionModel.predict_many: grouped towers and decodes) on fresh batch
    # objects: the same answers as the oracle's
    fresh = [dict(b, image=b["image"].view_as(b["image"])) for b in batches]
    with torch.no_grad():
        assert list(model.predict_many(fresh, eos_stop=False)) == want
