"""GPU parity: libmpr kernels (through the C ABI) vs the CPU oracle on seeded inputs.

Tolerances (fp32 everywhere; only the summation order differs from the CPU reference):
* retrieval ids: bit-exact; distances rel 2e-5.
* encoder / T5 float outputs: max|gpu - cpu| <= FP_TOL * max|cpu|.
"""
import numpy as np
import pytest
import torch

from multimodalpromptretrieval_amd import synthetic as syn
from oracle import clip as oclip
from oracle import retrieval as oret
from oracle import t5 as ot5

pytestmark = pytest.mark.gpu
FP_TOL = 2e-4
DIST_RTOL = 2e-5


def _rel_err(a: torch.Tensor, b: torch.Tensor) -> float:
    a = a.detach().float().cpu()
    b = b.detach().float().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp(min=1e-30))


@pytest.fixture(scope="module")
def index_mod():
    from multimodalpromptretrieval_amd import index
    return index


@pytest.mark.parametrize("n,d,b,k", [(6500, 1024, 16, 1), (6500, 1024, 16, 3),
                                     (6500, 1024, 16, 5), (10000, 1024, 16, 15),
                                     (512, 512, 33, 64), (7, 16, 3, 7), (65536, 1024, 16, 5),
                                     # large batches: the GEMM-shaped scan (b >= 64, k <= 16)
                                     (20000, 512, 256, 5), (5003, 1024, 64, 16),
                                     (999, 64, 100, 1), (70, 512, 300, 3),
                                     # b >= 64, d = 512, k 17..32: not coarse-eligible (its
                                     # gated exact fallback handles k <= 16 only)
                                     (20000, 512, 256, 20), (20000, 512, 128, 32)])
def test_scan_topk_l2(device, index_mod, n, d, b, k):
    X = syn.index_rows(1, n, d)
    q = syn.index_rows(2, b, d)
    ix = index_mod.DeviceIndex(X, device)
    dist, ids = ix.search(q.to(device), k)
    torch.cuda.synchronize()
    ref = oret.cdist(q, X)
    ref_ids = oret.topk_ids(ref, k, skip_first=False)
    assert torch.equal(ids.cpu(), ref_ids), "retrieved ids differ from the CPU reference"
    ref_d = torch.gather(ref, 1, ref_ids)
    assert torch.allclose(dist.cpu(), ref_d, rtol=DIST_RTOL, atol=1e-5)


def test_scan_ties_lowest_id(device, index_mod):
    # Integer-valued rows: every dot product is exact in any order, so duplicates tie exactly.
    g = np.random.Generator(np.random.PCG64(5))
    X = torch.from_numpy(g.integers(-3, 4, size=(300, 64)).astype(np.float32))
    X[[17, 101, 250]] = X[200].clone()  # exact duplicates of row 200
    q = X[[200, 5, 17]].clone()
    ix = index_mod.DeviceIndex(X, device)
    dist, ids = ix.search(q.to(device), 6)
    ref_ids = oret.topk_ids(oret.cdist(q, X), 6, skip_first=False)
    assert torch.equal(ids.cpu(), ref_ids)
    assert ids[0, :4].tolist() == [17, 101, 200, 250]


def test_scan_large_batch_ties_and_cosine(device, index_mod):
    """Large-batch path: exact duplicates resolve to the lowest id; cosine ids match too."""
    g = np.random.Generator(np.random.PCG64(9))
    X = torch.from_numpy(g.integers(-3, 4, size=(3000, 128)).astype(np.float32))
    X[[17, 1101, 2950]] = X[2000].clone()
    q = torch.cat([X[[2000, 5, 17]], torch.from_numpy(
        g.integers(-3, 4, size=(125, 128)).astype(np.float32))], 0)
    ix = index_mod.DeviceIndex(X, device)
    dist, ids = ix.search(q.to(device), 6)
    ref_ids = oret.topk_ids(oret.cdist(q, X), 6, skip_first=False)
    assert torch.equal(ids.cpu(), ref_ids)
    assert ids[0, :4].tolist() == [17, 1101, 2000, 2950]
    Xc = syn.index_rows(3, 4000, 512)
    qc = syn.index_rows(4, 96, 512)
    ixc = index_mod.DeviceIndex(Xc, device, metric=index_mod.COSINE)
    sim, idc = ixc.search(qc.to(device), 5)
    ref_idc, ref_sim = oret.cosine_topk(qc, Xc, 5)
    assert torch.equal(idc.cpu(), ref_idc)
    assert torch.allclose(sim.cpu(), ref_sim, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("b", [96, 256])
def test_coarse_path_ties_lowest_id(device, index_mod, b):
    """The coarse bf16 path (L2, d = 512, b >= 64): exact duplicates resolve to the lowest id,
    as in the exact scans.  Small-integer rows make every dot product exact in bf16 and in any
    fp32 summation order, so the coarse keys, the re-rank and the reference all tie exactly."""
    g = np.random.Generator(np.random.PCG64(19))
    n = 20000
    X = torch.from_numpy(g.integers(-3, 4, size=(n, 512)).astype(np.float32))
    X[[40, 9001, 19999]] = X[12345].clone()
    q = torch.from_numpy(g.integers(-3, 4, size=(b, 512)).astype(np.float32))
    q[0] = X[12345]
    q[1] = X[12345] + 1.0          # all four duplicates tie at the same nonzero distance
    ix = index_mod.DeviceIndex(X, device)
    dist, ids = ix.search(q.to(device), 5)
    ref_ids = oret.topk_ids(oret.cdist(q, X), 5, skip_first=False)
    assert torch.equal(ids.cpu(), ref_ids)
    assert ids[0, :4].tolist() == [40, 9001, 12345, 19999]
    assert ids[1, :4].tolist() == [40, 9001, 12345, 19999]


def test_scan_cosine(device, index_mod):
    X = syn.index_rows(3, 5000, 512)
    q = syn.index_rows(4, 16, 512)
    ix = index_mod.DeviceIndex(X, device, metric=index_mod.COSINE)
    sim, ids = ix.search(q.to(device), 5)
    ref_ids, ref_sim = oret.cosine_topk(q, X, 5)
    assert torch.equal(ids.cpu(), ref_ids)
    assert torch.allclose(sim.cpu(), ref_sim, rtol=1e-5, atol=1e-6)


def test_scan_scores_matrix(device, index_mod):
    X = syn.index_rows(6, 1000, 1024)
    q = syn.index_rows(7, 20, 1024)
    ix = index_mod.DeviceIndex(X, device)
    s = ix.scores(q.to(device))
    assert _rel_err(s, oret.cdist(q, X)) < 1e-5


def test_topk_merge_shards(device, index_mod):
    X = syn.index_rows(8, 4000, 1024)
    q = syn.index_rows(9, 16, 1024)
    shards = [index_mod.DeviceIndex(X[i * 1000:(i + 1) * 1000], device, row_offset=i * 1000)
              for i in range(4)]
    parts = [s.search(q.to(device), 5) for s in shards]
    cd = torch.cat([p[0] for p in parts], 1)
    ci = torch.cat([p[1] for p in parts], 1)
    d, ids = index_mod.topk_merge(cd, ci, 5)
    ref_ids = oret.topk_ids(oret.cdist(q, X), 5, False)
    assert torch.equal(ids.cpu(), ref_ids)


@pytest.mark.parametrize("k", [5, 100])
def test_topk_merge_fewer_valid_than_k(device, index_mod, k):
    """Candidate lists whose valid entries (id >= 0) number fewer than k (tiny shards pad with
    -1 sentinels): the valid ones come first in order, the remaining ranks are NaN / -1 — for
    the wave merge (k <= 64) and the radix select (k > 64)."""
    g = torch.Generator().manual_seed(3)
    b, n = 6, 160
    cd = torch.rand((b, n), generator=g)
    ci = torch.arange(n, dtype=torch.int64).repeat(b, 1)
    nvalid = [0, 1, 3, k - 1, min(k, n), n][:b]
    for r, nv in enumerate(nvalid):
        ci[r, nv:] = -1
        cd[r, nv:] = float("inf")
    d, ids = index_mod.topk_merge(cd.to(device), ci.to(device), k)
    d, ids = d.cpu(), ids.cpu()
    for r, nv in enumerate(nvalid):
        m = min(nv, k)
        order = torch.argsort(cd[r, :nv], stable=True)[:m]
        assert torch.equal(ids[r, :m], order), r
        assert torch.equal(d[r, :m], cd[r, order]), r
        assert bool((ids[r, m:] == -1).all()) and bool(torch.isnan(d[r, m:]).all()), r


@pytest.mark.parametrize("W,Bp,b,kc,k,metric", [(8, 256, 256, 5, 5, 0), (3, 20, 16, 4, 4, 0),
                                                 (2, 17, 5, 15, 15, 1), (8, 16, 16, 64, 64, 0)])
def test_topk_merge_packed_equals_unpacked(device, index_mod, W, Bp, b, kc, k, metric):
    """mpr_topk_pack + mpr_topk_merge_packed (the sharded search's exchange, merged as it
    arrives: [W][Bp][kc][2] float64) give topk_merge's outputs over the unpacked [b, W kc]
    lists, exact ties (duplicated keys across shards) and -1 / NaN empty slots included."""
    from multimodalpromptretrieval_amd import _lib
    g = torch.Generator().manual_seed(W * 100 + kc)
    d = torch.rand((W, Bp, kc), generator=g)
    d[1 % W, :, 0] = d[0, :, 0]                      # exact ties across shards
    ids = torch.randint(0, 1 << 30, (W, Bp, kc), generator=g)
    ids[0, 0, -1] = -1                               # an empty slot (tiny shard)
    d[0, 0, -1] = float("nan")
    dd, ii = d.to(device).contiguous(), ids.to(device).contiguous()
    packed = torch.empty((W, Bp, kc, 2), device=device, dtype=torch.float64)
    _lib.call("mpr_topk_pack", _lib.ptr(dd), _lib.ptr(ii), dd.numel(), _lib.ptr(packed),
              _lib.stream_ptr(device))
    assert torch.equal(packed[..., 0].cpu().nan_to_num(-7.0), d.double().nan_to_num(-7.0))
    assert torch.equal(packed[..., 1].cpu(), ids.double())
    od = torch.empty((b, k), device=device)
    oi = torch.empty((b, k), device=device, dtype=torch.int64)
    _lib.call("mpr_topk_merge_packed", _lib.ptr(packed), W, Bp, b, kc, k, metric, _lib.ptr(od),
              _lib.ptr(oi), _lib.stream_ptr(device))
    cd = dd[:, :b].permute(1, 0, 2).reshape(b, W * kc).contiguous()
    ci = ii[:, :b].permute(1, 0, 2).reshape(b, W * kc).contiguous()
    rd, ri = index_mod.topk_merge(cd, ci, k, metric)
    assert torch.equal(oi.cpu(), ri.cpu())
    assert torch.equal(od.cpu().nan_to_num(-7.0), rd.cpu().nan_to_num(-7.0))


@pytest.fixture(scope="module")
def clip_sd():
    return syn.clip_state_dict(11)


def test_vit_cls_and_tokens(device, clip_sd):
    from multimodalpromptretrieval_amd.encoders import CLS, TOKENS, DeviceViT
    vit = DeviceViT(clip_sd, device)
    img = syn.images(12, 4)
    cls = vit(img.to(device), CLS)
    tok = vit(img.to(device), TOKENS)
    assert _rel_err(cls, oclip.encode_image(clip_sd, img)) < FP_TOL
    assert _rel_err(tok, oclip.image_token_features(clip_sd, img)) < FP_TOL


def test_vit_pair_matches_single(device, clip_sd):
    """Paired pass (two towers, shared launches) == two single calls, bit for bit."""
    from multimodalpromptretrieval_amd.encoders import CLS, TOKENS, DeviceViT
    a = DeviceViT(clip_sd, device)
    b = DeviceViT(syn.clip_state_dict(14), device)
    img = syn.images(15, 16).to(device)
    cls, tok = a.forward_pair(b, img, CLS, TOKENS)
    assert torch.equal(cls, a(img, CLS)) and torch.equal(tok, b(img, TOKENS))
    tok2, cls2 = b.forward_pair(a, img[:3], TOKENS, CLS)
    assert torch.equal(cls2, a(img[:3], CLS)) and torch.equal(tok2, b(img[:3], TOKENS))
    # determinism of grouped launches (a stage-reuse race once made ~3% of them differ)
    for _ in range(12):
        c_i, t_i = a.forward_pair(b, img, CLS, TOKENS)
        assert torch.equal(c_i, cls) and torch.equal(t_i, tok)


_POOL_SCRIPT = r"""
import sys, torch
sys.path.insert(0, {root!r})
from multimodalpromptretrieval_amd import synthetic as syn
from multimodalpromptretrieval_amd.encoders import CLS, TOKENS, DeviceCLIPText, DeviceViT
dev = torch.device("cuda:0")
sd = syn.clip_state_dict(11)
vit, txt = DeviceViT(sd, dev), DeviceCLIPText(sd, dev)
img = syn.images(15, 16).to(dev)
toks = syn.clip_tokens(17, 16)
torch.save({{"cls": vit(img, CLS).cpu(), "tok": vit(img, TOKENS).cpu(),
             "txt": txt(toks).cpu()}}, {out!r})
"""


def test_pooled_last_block_matches_full(device, clip_sd, tmp_path):
    """The pooled towers' last block over the CLS / EOT rows only (TowerRun::pool) == the block
    over every row (MPR_POOL_LAST=0, a fresh process), bit for bit; the CLS embedding is row 0
    of the token features of the same weights."""
    import os
    import subprocess
    import sys
    from multimodalpromptretrieval_amd.encoders import CLS, TOKENS, DeviceCLIPText, DeviceViT
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = str(tmp_path / "full.pt")
    env = dict(os.environ, MPR_POOL_LAST="0")
    subprocess.run([sys.executable, "-c", _POOL_SCRIPT.format(root=root, out=out)], env=env,
                   check=True, timeout=240)
    full = torch.load(out, weights_only=True)
    vit, txt = DeviceViT(clip_sd, device), DeviceCLIPText(clip_sd, device)
    img = syn.images(15, 16).to(device)
    toks = syn.clip_tokens(17, 16)
    cls, tok, tt = vit(img, CLS).cpu(), vit(img, TOKENS).cpu(), txt(toks).cpu()
    assert torch.equal(cls, full["cls"]) and torch.equal(tt, full["txt"])
    assert torch.equal(tok, full["tok"])
    assert torch.equal(cls, tok[:, 0])


def test_encode_towers_matches_separate(device, clip_sd):
    """ViT pair + text tower in one lockstep pass == the three separate calls, bit for bit."""
    from multimodalpromptretrieval_amd.encoders import (CLS, TOKENS, DeviceCLIPText, DeviceViT,
                                                         encode_towers)
    a, b = DeviceViT(clip_sd, device), DeviceViT(syn.clip_state_dict(14), device)
    txt = DeviceCLIPText(clip_sd, device)
    img = syn.images(16, 16).to(device)
    toks = syn.clip_tokens(17, 16)
    ca, tb, tt = encode_towers(a, img, CLS, vit_b=b, mode_b=TOKENS, text=txt, tokens=toks)
    assert torch.equal(ca, a(img, CLS)) and torch.equal(tb, b(img, TOKENS))
    assert torch.equal(tt, txt(toks))
    ca1, _, tt1 = encode_towers(a, img[:5], CLS, text=txt, tokens=toks[:5])
    assert torch.equal(ca1, a(img[:5], CLS)) and torch.equal(tt1, txt(toks[:5]))
    _, _, t_only = encode_towers(text=txt, tokens=toks[:3])
    assert torch.equal(t_only, txt(toks[:3]))


def test_encode_towers_multi_matches_per_batch(device, clip_sd):
    """Two batches' towers in one pass (images concatenated for the ViTs, each batch's questions
    a text run of its own length) == the per-batch passes, bit for bit."""
    from multimodalpromptretrieval_amd.encoders import (CLS, TOKENS, DeviceCLIPText, DeviceViT,
                                                         encode_towers, encode_towers_multi)
    a, b = DeviceViT(clip_sd, device), DeviceViT(syn.clip_state_dict(14), device)
    txt = DeviceCLIPText(clip_sd, device)
    imgs = [syn.images(60, 11).to(device), syn.images(61, 11).to(device)]
    toks = [syn.clip_tokens(62, 11), syn.clip_tokens(63, 11).clone()]
    eot = int(toks[1].max())
    toks[1][:, 9] = eot  # the second batch's prompts end earlier: a shorter text run
    toks[1][:, 10:] = 0
    assert int(toks[0].argmax(1).max()) != int(toks[1].argmax(1).max())
    want = [encode_towers(a, imgs[i], CLS, vit_b=b, mode_b=TOKENS, text=txt, tokens=toks[i])
            for i in range(2)]
    ca, tb, tts = encode_towers_multi(a, torch.cat(imgs), CLS, vit_b=b, mode_b=TOKENS, text=txt,
                                      tokens=toks)
    # 11-image batches: alone some projections take the 32x32 tile that 22 images' rows would
    # not; the per-batch tile choice keeps the pass bit-identical
    assert torch.equal(ca[:11], want[0][0]) and torch.equal(ca[11:], want[1][0])
    assert torch.equal(tb[:11], want[0][1]) and torch.equal(tb[11:], want[1][1])
    assert torch.equal(tts[0], want[0][2]) and torch.equal(tts[1], want[1][2])
    with pytest.raises(ValueError):  # unequal batches cannot share a pass
        encode_towers_multi(a, torch.cat([imgs[0], imgs[1][:5]]), CLS, text=txt,
                            tokens=[toks[0], toks[1][:5]])


def test_tower_graphs_match_eager(device, clip_sd, monkeypatch):
    """MPR_TOWER_GRAPHS=1: a tower pass captured into a hipGraph over staged inputs / outputs
    (first sighting eager + capture, then replays) gives the eager pass's outputs bit for bit,
    for strided outputs (the retrieval's [img | txt] query rows) and a new shape."""
    from multimodalpromptretrieval_amd.encoders import (CLS, TOKENS, DeviceCLIPText, DeviceViT,
                                                         encode_towers_multi)
    a, b = DeviceViT(clip_sd, device), DeviceViT(syn.clip_state_dict(14), device)
    txt = DeviceCLIPText(clip_sd, device)
    imgs = torch.cat([syn.images(70, 8), syn.images(71, 8)]).to(device)
    toks = [syn.clip_tokens(72, 8), syn.clip_tokens(73, 8)]

    def run():
        q = torch.full((16, 1024), float("nan"), device=device)
        _, tb, _ = encode_towers_multi(a, imgs, CLS, out_a=q, out_a_bstride=1024, vit_b=b,
                                       mode_b=TOKENS, text=txt, tokens=toks,
                                       out_t=[q[:8, 512:], q[8:, 512:]],
                                       out_t_bstride=[1024, 1024])
        torch.cuda.synchronize()
        return q.cpu(), tb.cpu()

    monkeypatch.delenv("MPR_TOWER_GRAPHS", raising=False)
    want_q, want_t = run()
    monkeypatch.setenv("MPR_TOWER_GRAPHS", "1")
    for _ in range(3):  # eager + capture, then graph replays
        q, t = run()
        assert torch.equal(q, want_q) and torch.equal(t, want_t)
    toks[1] = toks[1].clone()
    toks[1][:, 5:] = 0
    toks[1][:, 4] = int(toks[0].max())       # a shorter text run: a new shape
    monkeypatch.delenv("MPR_TOWER_GRAPHS", raising=False)
    want_q, want_t = run()
    monkeypatch.setenv("MPR_TOWER_GRAPHS", "1")
    for _ in range(2):
        q, t = run()
        assert torch.equal(q, want_q) and torch.equal(t, want_t)


def test_encode_towers_slots_run_concurrently(device, clip_sd):
    """Two batches' lockstep passes on workspace slots 0 and 1 on two streams at once (repeated,
    so the passes overlap): each equals its pass run alone, bit for bit."""
    from multimodalpromptretrieval_amd.encoders import CLS, TOKENS, DeviceCLIPText, DeviceViT, \
        encode_towers
    a, b = DeviceViT(clip_sd, device), DeviceViT(syn.clip_state_dict(14), device)
    txt = DeviceCLIPText(clip_sd, device)
    imgs = [syn.images(30 + i, 16).to(device) for i in range(2)]
    toks = [syn.clip_tokens(40 + i, 16) for i in range(2)]
    want = [encode_towers(a, imgs[i], CLS, vit_b=b, mode_b=TOKENS, text=txt, tokens=toks[i])
            for i in range(2)]
    streams = [torch.cuda.Stream(device) for _ in range(2)]
    for _ in range(4):
        got = []
        for i, st in enumerate(streams):
            st.wait_stream(torch.cuda.current_stream(device))
            with torch.cuda.stream(st):
                got.append(encode_towers(a, imgs[i], CLS, vit_b=b, mode_b=TOKENS, text=txt,
                                         tokens=toks[i], slot=i))
        for st in streams:
            torch.cuda.current_stream(device).wait_stream(st)
        for g, w in zip(got, want):
            assert all(torch.equal(x, y) for x, y in zip(g, w))
    with pytest.raises(RuntimeError):
        encode_towers(a, imgs[0], CLS, slot=4)


def test_create_retrieval_dataset_builds_and_caches(device, clip_sd, tmp_path):
    """Index build (dataset/VQAFeatureDataset.py:118-185): the rows are
    each batch's encode_queries rows bit for bit and the oracle towers' rows within FP_TOL at full
    ViT-B/32 + CLIP-text size (the reference's own rows at G2 size: test_gpu_dropin.py), the lists
    follow the loader, the second call
    loads the cache (safe formats) instead of encoding, and a query finds its own row."""
    from multimodalpromptretrieval_amd.dataset import VQARetrieval
    r = VQARetrieval(device, clip_state_dict=clip_sd, clip_tokenizer=syn.hash_clip_tokenize)
    loader = []
    for i, b in enumerate((5, 7, 3)):
        loader.append({"image": syn.images(50 + i, b).to(device),
                       "question": [f"what organ is shown {i} {j}" for j in range(b)],
                       "answer": [f"a{i}{j}" for j in range(b)],
                       "question_type": ["organ"] * b,
                       "question_id": [f"{i}-{j}" for j in range(b)]})
    want = torch.cat([r.encode_queries(bt).cpu() for bt in loader])
    r.create_retrieval_dataset(loader, is_training_phase=False, retrieval_k=1,
                               cache_dir=str(tmp_path))
    assert torch.equal(r.retrieval_embeddings.cpu(), want)
    # against the oracle's CLIP towers over the same loader (:145-148: [image CLS ‖ text EOT])
    oracle_rows = torch.cat([torch.cat([oclip.encode_image(clip_sd, bt["image"].cpu()),
                                        oclip.encode_text(clip_sd,
                                                          syn.hash_clip_tokenize(bt["question"]))],
                                       1) for bt in loader])
    assert _rel_err(r.retrieval_embeddings.cpu(), oracle_rows) < FP_TOL
    assert r.retrieval_answers == [a for bt in loader for a in bt["answer"]]
    assert r.retrieval_question_info["question_id"] == [q for bt in loader
                                                          for q in bt["question_id"]]
    r2 = VQARetrieval(device, clip_state_dict=clip_sd, clip_tokenizer=syn.hash_clip_tokenize)
    r2.encode_queries = None  # a cache hit must not encode
    r2.create_retrieval_dataset(loader, is_training_phase=False, retrieval_k=1,
                                cache_dir=str(tmp_path))
    assert torch.equal(r2.retrieval_embeddings.cpu(), want)
    got = r.retrieve_closest_qa_pairs(loader[1], return_ans=True)
    assert got == [[a] for a in loader[1]["answer"]]
    # equal-sized batches share one tower pass: still each batch's rows bit for bit
    loader2 = [dict(bt, image=syn.images(60 + i, 4).to(device),
                    question=[f"which plane {i} {j}" for j in range(4)],
                    answer=[f"p{i}{j}" for j in range(4)], question_type=["plane"] * 4,
                    question_id=[f"p{i}-{j}" for j in range(4)]) for i, bt in enumerate(loader)]
    want2 = torch.cat([r.encode_queries(bt).cpu() for bt in loader2])
    r.create_retrieval_dataset(loader2, is_training_phase=False, retrieval_k=1,
                               cache_dir=str(tmp_path / "two"))
    assert torch.equal(r.retrieval_embeddings.cpu(), want2)
    assert r.retrieval_answers == [a for bt in loader2 for a in bt["answer"]]


def test_clip_text(device, clip_sd):
    from multimodalpromptretrieval_amd.encoders import DeviceCLIPText
    txt = DeviceCLIPText(clip_sd, device)
    toks = syn.clip_tokens(13, 5)
    out = txt(toks)
    assert _rel_err(out, oclip.encode_text(clip_sd, toks)) < FP_TOL
    full = txt(toks.to(device))  # device tokens: all 77 positions, same pooled result
    assert _rel_err(full, out) < 1e-5


@pytest.fixture(scope="module")
def t5_sd():
    return syn.t5_state_dict(21)


def _t5_inputs(b=4, seed=22):
    ids, mask = syn.t5_prompt_ids(seed, b)
    sd_img = syn.images(seed, b)  # noqa: F841  (image tokens come from a random tensor here)
    g = torch.Generator().manual_seed(seed)
    img_tok = torch.randn(b, 50, 512, generator=g) * 0.5
    return ids, mask, img_tok


def test_t5_encode_logits_generate(device, t5_sd):
    from multimodalpromptretrieval_amd.t5 import DeviceT5
    m = DeviceT5(t5_sd, device)
    ids, mask, img_tok = _t5_inputs()
    B = ids.shape[0]
    emb = torch.cat([img_tok, t5_sd["shared.weight"][ids]], 1)
    full_mask = torch.cat([torch.ones(B, 50, dtype=torch.long), mask], 1)
    enc = m.encode(emb, full_mask)
    ref_enc = ot5.encode(t5_sd, emb, full_mask, 8)
    assert _rel_err(enc, ref_enc) < FP_TOL
    dec_in = torch.randint(0, 32100, (B, 7), generator=torch.Generator().manual_seed(3))
    lg = m.logits(emb, full_mask, dec_in)
    ref_lg = ot5.decoder_logits(t5_sd, ref_enc, full_mask, dec_in, 8)
    assert _rel_err(lg, ref_lg) < FP_TOL
    toks = m.generate(emb, full_mask, max_new_tokens=20)
    ref_toks, step_logits = ot5.generate(t5_sd, emb, full_mask, 8, 20)
    # greedy ids per row up to (and including) that row's first step whose reference top-2
    # margin is within the fp tolerance (past a near-tie the two greedy paths may fork)
    margins = torch.stack([s.topk(2).values[:, 0] - s.topk(2).values[:, 1]
                           for s in step_logits], 1)            # [B, steps]
    # (column 0 is the decoder start token; step s's token is column s + 1)
    compared = 0
    for r in range(B):
        close = (margins[r] <= 1e-3).nonzero()
        n = int(close[0]) if len(close) else margins.shape[1]
        assert torch.equal(toks[r, :n + 1], ref_toks[r, :n + 1]), r
        compared += n
    assert compared > 0


def test_t5_generate_graph_replay_matches_eager(device, t5_sd, monkeypatch):
    from multimodalpromptretrieval_amd.t5 import DeviceT5
    m = DeviceT5(t5_sd, device)
    ids, mask, img_tok = _t5_inputs(5, 41)
    emb = torch.cat([img_tok, t5_sd["shared.weight"][ids]], 1).to(device)
    fm = torch.cat([torch.ones(5, 50, dtype=torch.long), mask], 1).to(device)
    a = m.generate_padded(emb, fm, 20).cpu()        # captured + replayed
    b = m.generate_padded(emb, fm, 20).cpu()        # graph cache hit
    monkeypatch.setenv("MPR_GRAPHS", "0")
    c = m.generate_padded(emb, fm, 20).cpu()        # eager launches
    assert torch.equal(a, b) and torch.equal(a, c)
    d = m.generate_padded(emb[:3], fm[:3], 7).cpu() # another shape
    assert torch.equal(d, c[:3, :8])


def test_t5_generate_on_decode_stream(device, t5_sd):
    """Decode loop on a CU-partition stream: same tokens as on the caller's stream."""
    from multimodalpromptretrieval_amd import _lib
    from multimodalpromptretrieval_amd.t5 import DeviceT5
    m = DeviceT5(t5_sd, device)
    ids, mask, img_tok = _t5_inputs(6, 43)
    emb = torch.cat([img_tok, t5_sd["shared.weight"][ids]], 1).to(device)
    fm = torch.cat([torch.ones(6, 50, dtype=torch.long), mask], 1).to(device)
    a = m.generate_padded(emb, fm, 20).cpu()
    m.set_decode_stream(_lib.role_stream(device, "decode"))
    b = m.generate_padded(emb, fm, 20).cpu()
    c = m.generate_padded(emb[:2], fm[:2], 20).cpu()
    m.set_decode_stream(None)
    assert torch.equal(a, b) and torch.equal(c, a[:2])


def _t5_batch(t5_sd, b, seed, extra=0):
    ids, mask, img_tok = _t5_inputs(b, seed)
    if extra:  # a longer prompt (another length bucket): trailing padding tokens, mask 0
        ids = torch.cat([ids, torch.zeros(b, extra, dtype=ids.dtype)], 1)
        mask = torch.cat([mask, torch.zeros(b, extra, dtype=mask.dtype)], 1)
    emb = torch.cat([img_tok, t5_sd["shared.weight"][ids]], 1)
    fm = torch.cat([torch.ones(b, 50, dtype=torch.long), mask], 1)
    return emb, fm


@pytest.mark.parametrize("graphs", ["1", "0"])
def test_t5_generate_pair_matches_single(device, t5_sd, monkeypatch, graphs):
    """Two to four batches through one shared decode loop (up to 64 rows: the two- and
    four-row-group skinny GEMMs, the 64-row greedy step): each batch's tokens are bit-identical
    to its own generate, with equal and different source-length buckets, any batch the longest,
    16 + 16 rows, and an empty second batch."""
    from multimodalpromptretrieval_amd.t5 import DeviceT5
    monkeypatch.setenv("MPR_GRAPHS", graphs)
    m = DeviceT5(t5_sd, device)
    A = _t5_batch(t5_sd, 7, 61)
    B = _t5_batch(t5_sd, 9, 62, extra=19)
    C = _t5_batch(t5_sd, 16, 63)
    D = _t5_batch(t5_sd, 16, 64, extra=8)
    single = {k: m.generate_padded(*v, 20).cpu() for k, v in
              {"A": A, "B": B, "C": C, "D": D}.items()}
    assert A[0].shape[1] != B[0].shape[1]
    for x, y in (("A", "B"), ("B", "A"), ("C", "D"), ("A", "A")):
        va, vb = {"A": A, "B": B, "C": C, "D": D}[x], {"A": A, "B": B, "C": C, "D": D}[y]
        oa, ob = m.generate_pair_padded(*va, *vb, 20, slot=1)
        assert torch.equal(oa.cpu(), single[x]), (x, y)
        assert torch.equal(ob.cpu(), single[y]), (x, y)
    e = (A[0][:0], A[1][:0])
    oa, ob = m.generate_pair_padded(*A, *e, 20)
    assert torch.equal(oa.cpu(), single["A"]) and ob.shape == (0, 21)
    oa, ob = m.generate_pair_padded(*B, *A, 5, slot=2)  # fewer steps: a prefix of the same greedy run
    assert torch.equal(oa.cpu(), single["B"][:, :6]) and torch.equal(ob.cpu(), single["A"][:, :6])
    # 3 and 4 batches in one loop (48 / 57 rows: the four-row-group GEMVs, a 64-row greedy step)
    named = {"A": A, "B": B, "C": C, "D": D}
    for keys in ("ACD", "CDAB", "BDCA"):
        outs = m.generate_batches_padded([named[k] for k in keys], 20, slot=3)
        for k, o in zip(keys, outs):
            assert torch.equal(o.cpu(), single[k]), (keys, k)
    outs = m.generate_batches_padded([named[k] for k in "ABCDDCBA"], 20, slot=3)  # 114 rows
    for k, o in zip("ABCDDCBA", outs):
        assert torch.equal(o.cpu(), single[k]), ("ABCDDCBA", k)
    with pytest.raises(ValueError):  # at most 16 batches (256 rows) per decode loop
        m.generate_batches_padded([A, B, C, D] * 4 + [A], 20)
    # a batch of more than 16 rows runs as 16-row chunks (here 16 + 8): each row as alone
    big = (torch.cat([C[0], A[0][:8]]), torch.cat([C[1], A[1][:8]])) if C[0].shape[1] == \
        A[0].shape[1] else (torch.cat([C[0], C[0][:8]]), torch.cat([C[1], C[1][:8]]))
    want_big = torch.cat([m.generate_padded(big[0][:16], big[1][:16], 20).cpu(),
                          m.generate_padded(big[0][16:], big[1][16:], 20).cpu()])
    assert torch.equal(m.generate_padded(*big, 20).cpu(), want_big)


def test_t5_generate_over_128_rows_two_slots(device, t5_sd, monkeypatch):
    """More than 128 rows (config C5's 256 questions): the 128-row decode loops run on two
    slots and streams at once; tokens equal the one-slot sequential run bit for bit."""
    from multimodalpromptretrieval_amd.t5 import DeviceT5
    m = DeviceT5(t5_sd, device)
    A = _t5_batch(t5_sd, 16, 71)
    emb = torch.cat([A[0]] * 12 + [A[0][:5]])   # 197 rows: loops of 128 + 69
    emb = emb + 1e-3 * torch.randn(emb.shape, generator=torch.Generator().manual_seed(5))
    fm = torch.cat([A[1]] * 12 + [A[1][:5]])
    monkeypatch.setenv("MPR_SPLIT_SLOTS", "0")
    want = m.generate_padded(emb, fm, 20).cpu()
    monkeypatch.setenv("MPR_SPLIT_SLOTS", "1")
    got = m.generate_padded(emb, fm, 20).cpu()
    assert got.shape == (197, 21)
    assert torch.equal(got, want)


@pytest.fixture(scope="module")
def grouped_40(t5_sd):
    """40 distinct prompts (three 16-row groups sharing one decode loop) and the oracle's greedy
    ids and per-step logits for them."""
    ids, mask, img_tok = _t5_inputs(40, 61)
    emb = torch.cat([img_tok, t5_sd["shared.weight"][ids]], 1)
    fm = torch.cat([torch.ones(40, 50, dtype=torch.long), mask], 1)
    ref_toks, step_logits = ot5.generate(t5_sd, emb, fm, 8, 20)
    return emb, fm, ref_toks, step_logits


@pytest.mark.parametrize("tiled", ["1", "0"])
def test_t5_grouped_decode_head_vs_oracle(device, t5_sd, grouped_40, monkeypatch, tiled):
    """The argmax head of a decode over > 32 rows: RMSNorm + the tiled GEMM + a row argmax
    (MPR_TILED_HEAD=1, the default from d >= 768) or the skinny GEMV (0), on the 8-launch chain
    (MPR_DECODE_FOLD=0: this t5-small model would otherwise take the folded chain, whose head is
    the skinny GEMV).  Greedy ids equal the oracle's per row up to (and including) its first
    step with a top-2 margin <= 1e-3."""
    from multimodalpromptretrieval_amd.t5 import DeviceT5
    monkeypatch.setenv("MPR_TILED_HEAD", tiled)
    monkeypatch.setenv("MPR_DECODE_FOLD", "0")
    m = DeviceT5(t5_sd, device)
    emb, fm, ref_toks, step_logits = grouped_40
    toks = m.generate_padded(emb, fm, 20).cpu().long()
    margins = torch.stack([s.topk(2).values[:, 0] - s.topk(2).values[:, 1]
                           for s in step_logits], 1)
    compared = 0
    for r in range(emb.shape[0]):
        close = (margins[r] <= 1e-3).nonzero()
        n = int(close[0]) if len(close) else margins.shape[1]
        assert torch.equal(toks[r, :n + 1], ref_toks[r, :n + 1]), r
        compared += n
    assert compared > 200


@pytest.mark.parametrize("text_only", [False, True])
def test_decode_attention_wave_form_matches_block(device, t5_sd, monkeypatch, text_only):
    """Decodes over >= 64 rows (>= 512 batch x head pairs) run the decode attention one wave per
    pair (attention_decode_wave_kernel), whose outputs are bit-identical to the block kernel's
    (MPR_ATT_WAVE=0), and pairs with 65..128 keys (this cross-attention over 73 source rows) two
    waves per pair (attention_decode_wave2_kernel; MPR_ATT_WAVE2=0 keeps one): the greedy tokens
    of 128 + 69 rows are equal in all three forms.  At <= 64 keys (the self-attentions; the
    cross-attention over the text-only prompts, <= 31 source rows) the one-wave form is the
    single-half instantiation (MPR_ATT_KEYS64=0 keeps the two-half code): equal tokens too."""
    from multimodalpromptretrieval_amd.t5 import DeviceT5
    A = _t5_batch(t5_sd, 16, 73)
    if text_only:  # no 50 image-token prefix: the cross-attention takes <= 64 keys
        A = (A[0][:, 50:].contiguous(), A[1][:, 50:].contiguous())
    emb = torch.cat([A[0]] * 12 + [A[0][:5]])
    emb = emb + 1e-3 * torch.randn(emb.shape, generator=torch.Generator().manual_seed(6))
    fm = torch.cat([A[1]] * 12 + [A[1][:5]])
    monkeypatch.setenv("MPR_ATT_WAVE", "0")
    want = DeviceT5(t5_sd, device).generate_padded(emb, fm, 20).cpu()
    monkeypatch.setenv("MPR_ATT_WAVE", "1")
    got = DeviceT5(t5_sd, device).generate_padded(emb, fm, 20).cpu()
    assert torch.equal(got, want)
    monkeypatch.setenv("MPR_ATT_WAVE2", "0")
    one_wave = DeviceT5(t5_sd, device).generate_padded(emb, fm, 20).cpu()
    assert torch.equal(one_wave, want)
    monkeypatch.setenv("MPR_ATT_KEYS64", "0")
    two_half = DeviceT5(t5_sd, device).generate_padded(emb, fm, 20).cpu()
    assert torch.equal(two_half, want)


@pytest.mark.parametrize("fold,text_only", [("1", False), ("0", False), ("1", True)])
def test_decode_attention_small_forms_match_block(device, t5_sd, monkeypatch, fold, text_only):
    """A one-batch decode (16 rows: 128 batch x head pairs) runs its attention a block of one wave
    per pair (attention_decode_wave1_kernel, default), two waves per pair past 64 keys
    (MPR_ATT_SMALL=wave2) or the 256-thread block kernel (block): greedy tokens equal in all
    three, on the folded and the 8-launch chain (73 source keys: the cross-attention takes both
    halves; text-only prompts: one; MPR_ATT_KEYS64 does not change this form)."""
    from multimodalpromptretrieval_amd.t5 import DeviceT5
    monkeypatch.setenv("MPR_DECODE_FOLD", fold)
    emb, fm = _t5_batch(t5_sd, 16, 73)
    if text_only:
        emb, fm = emb[:, 50:].contiguous(), fm[:, 50:].contiguous()
    got = {}
    for form in ("block", "wave1", "wave2", "keys64off"):
        monkeypatch.setenv("MPR_ATT_SMALL", "wave1" if form == "keys64off" else form)
        monkeypatch.setenv("MPR_ATT_KEYS64", "0" if form == "keys64off" else "1")
        got[form] = DeviceT5(t5_sd, device).generate_padded(emb, fm, 20).cpu()
    assert all(torch.equal(got[f], got["block"]) for f in ("wave1", "wave2", "keys64off"))


def test_grouped_decode_row_blocks_match(device, monkeypatch):
    """A t5-base decode loop of more than 128 rows runs its GEMVs on 64-row blocks (MR = 4,
    2-chunk passes); the same rows decoded as loops of <= 128 rows (32-row blocks, 4-chunk
    passes; MPR_GEN_PIECES=8) give the same greedy tokens bit for bit: rows are independent and
    every accumulator chain keeps its chunk order."""
    from multimodalpromptretrieval_amd import synthetic as syn
    from multimodalpromptretrieval_amd.t5 import DeviceT5
    m = DeviceT5(syn.t5_state_dict(3, syn.T5_BASE), device)
    g = torch.Generator().manual_seed(11)
    rows, L = 200, 40
    emb = torch.randn((rows, L, syn.T5_BASE.d_model), generator=g) * 0.3
    mask = torch.ones((rows, L))
    mask[1::3, 30:] = 0
    monkeypatch.setenv("MPR_GEN_PIECES", "8")
    want = m.generate_padded(emb.to(device), mask.to(device), 20).cpu()
    monkeypatch.setenv("MPR_GEN_PIECES", "16")
    got = m.generate_padded(emb.to(device), mask.to(device), 20).cpu()
    assert torch.equal(got, want)


def test_t5_embed_and_loss(device, t5_sd):
    from multimodalpromptretrieval_amd.t5 import DeviceT5
    m = DeviceT5(t5_sd, device)
    ids, mask, img_tok = _t5_inputs(3, 31)
    out = torch.zeros(3, 50 + ids.shape[1], 512, device=device)
    m.embed(ids, out, row0=50)
    assert torch.equal(out[:, 50:].cpu(), t5_sd["shared.weight"][ids])
    logits = torch.randn(3, 5, 32101)
    labels = torch.randint(0, 32101, (3, 5))
    labels[0, 3:] = -100
    loss = m.loss(logits.to(device), labels)
    ref = ot5.lm_loss(logits, labels)
    assert abs(float(loss) - float(ref)) < 1e-5 * max(1.0, abs(float(ref)))
