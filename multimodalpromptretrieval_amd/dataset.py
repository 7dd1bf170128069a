"""Retrieval surface of the reference's VQADataset, on the MI355X.

``VQARetrieval`` carries the two methods the reference's ``main.py`` wires into the model
(dataset/VQAFeatureDataset.py:118-246):

* ``create_retrieval_dataset(data_loader, prefix, is_training_phase=True, retrieval_k=15,
  use_additional_data=False)`` — encodes every retrieval example as [CLS image ‖ EOT text]
  (fp32, D = 1024 for ViT-B/32) and keeps the index resident in HBM (sharded over the process
  group when one is given);
* ``retrieve_closest_qa_pairs(batch, return_ans=False, return_info=None, return_dists=False,
  use_quantifier=True)`` — same four return types, same vote/bucket prompt.

Differences, all deliberate: exact distance ties resolve to the lowest row id (the reference's
unstable argsort is order-undefined there); the index cache is written in safe
formats (tensor + JSON, no pickles) under a key that includes the dataset size (the reference's
class-name key collides, F9); ``use_additional_data`` merges question-info dicts instead of
calling ``.extend`` on a dict (F9).  One search serves the analytics calls that ``main.py --test``
makes on the same batch (F10): the last batch's top-k is reused while the batch is unchanged.
"""
from __future__ import annotations

import json
import os
import pickle

import numpy as np
import torch

from . import _lib
from .encoders import CLS, DeviceCLIPText, DeviceViT, encode_towers, encode_towers_multi  # noqa: F401,E501
from .index import L2, DeviceIndex
from .staging import to_device

BUCKETS = ["very unlikely", "unlikely", "maybe", "likely", "very likely", "certainly"]


def clip_package_tokenizer():
    """``clip.tokenize`` restated (tokenization.ClipBPE) on the installed openai package's own
    vocabulary file; None when the package is absent."""
    try:
        import clip
    except ImportError:
        return None
    from .tokenization import ClipBPE
    path = os.path.join(os.path.dirname(clip.__file__), "bpe_simple_vocab_16e6.txt.gz")
    return ClipBPE(path).tokenize if os.path.exists(path) else clip.tokenize


def _default_clip():
    try:
        import clip  # noqa: F401
    except ImportError as e:
        raise RuntimeError("openai `clip` is not installed: pass clip_state_dict= (and "
                           "clip_tokenizer=, default tokenization.clip_tokenize)") from e
    import clip
    model, _ = clip.load("ViT-B/32", device="cpu")
    return model.float().state_dict(), clip_package_tokenizer()


def vote_prompt(row: list, use_quantifier: bool = True) -> str:
    """dataset/VQAFeatureDataset.py:216-230."""
    counts: dict = {}
    for a in row:
        counts[a] = counts.get(a, 0) + 1
    pred = max(counts, key=counts.get)
    certainty = max(counts.values()) / sum(counts.values())
    if use_quantifier:
        return f"I believe the answer is {BUCKETS[int(certainty * (len(BUCKETS) - 1))]} {pred}"
    return f"The most frequent answer is {pred}"


class _DataOnlyUnpickler(pickle.Unpickler):
    """Reads pickles of plain containers only (lists, dicts, tuples, str, numbers): no global is
    ever resolved, so nothing in the file can run."""

    def find_class(self, module, name):
        raise pickle.UnpicklingError(f"{module}.{name}: only plain lists / dicts / strings are "
                                     f"read from an index cache")


def read_pickled_data(path):
    """The reference's answers.pkl / answer_types.pkl (dataset/VQAFeatureDataset.py:130-135):
    a list of answer strings / a dict of lists.  Refuses anything that needs a global."""
    with open(path, "rb") as f:
        return _DataOnlyUnpickler(f).load()


class VQARetrieval:
    """Retrieval index + CLIP query encoders on one GPU (or sharded over a process group)."""

    RECENT = 64  # searches kept per batch key (a serving loop ahead of main.py's analytics)
    BUILD_SLOTS = min(2, int(os.environ.get("MPR_BUILD_SLOTS", "2")))  # index build passes in flight

    def __init__(self, device="cuda", clip_state_dict: dict = None, clip_tokenizer=None,
                 metric: int = L2, group=None, max_batch: int = None):
        self.device = torch.device(device)
        _lib.ensure_device(self.device)
        if clip_state_dict is None:
            clip_state_dict, default_tok = _default_clip()
            clip_tokenizer = clip_tokenizer or default_tok
        if clip_tokenizer is None:
            # clip.tokenize's algorithm (tokenization.ClipBPE) on the openai vocabulary when the
            # package is installed, else on the same-format stand-in vocabulary
            from .tokenization import clip_tokenize
            clip_tokenizer = clip_package_tokenizer() or clip_tokenize
        self.clip_tokenize = clip_tokenizer
        self.image_encoder = DeviceViT(clip_state_dict, self.device)
        self.text_encoder = DeviceCLIPText(clip_state_dict, self.device)
        self.embed_dim = self.image_encoder.out_dim + self.text_encoder.out_dim
        self.metric = metric
        self.group = group
        self.max_batch = max_batch  # sharded index: fixed query-block size (no per-search sync)
        self.retrieval_k = 15
        self.is_training_phase = False
        self.index = None
        self.cache_enabled = True
        self._prefetched = {}  # serving-loop lookahead: batch key -> enqueued search (prefetch)
        self._cache_key = None
        self._cache_val = None
        self._cache_ref = None
        self._recent = {}  # the last RECENT searches by batch key (host top-k, image ref)

    # ---- encoding ------------------------------------------------------------------------------
    def _streams(self):
        """The retrieval stream (_lib.role_stream "encode:towers"; tower workspace slot 0)."""
        if not hasattr(self, "_s_img"):
            self._s_img = _lib.role_stream(self.device, "encode:towers")
        return self._s_img

    def _slot_stream(self, slot: int):
        """Stream of tower workspace slot `slot` (slot 0 = the retrieval stream, so that every
        use of a slot stays ordered on one stream)."""
        if slot == 0:
            return self._streams()
        if not hasattr(self, "_s_slot"):
            self._s_slot = {}
        if slot not in self._s_slot:
            self._s_slot[slot] = _lib.role_stream(self.device, f"encode:towers{slot}")
        return self._s_slot[slot]

    def _scan_stream(self):
        """Every prefetched search runs on the slot-0 stream (the index keeps one search
        workspace; one more stream would also alias a hardware queue, 4 per process)."""
        return self._streams()

    def encode_image_pair(self, batch, other_vit, other_mode: int):
        """Run this retrieval's query encoders (``encode_image`` on the batch's images and
        ``encode_text`` on its questions) together with a second ViT of the same geometry over
        the same images (T5VisionModel's token-feature tower): one lockstep pass over the three
        CLIP towers (``encoders.encode_towers``).  The query rows are kept for the next
        ``encode_queries(batch)`` of the same batch object; returns the other tower's output and
        the stream it is produced on (the caller waits on that stream before using it)."""
        s_img = self._streams()
        cur = torch.cuda.current_stream(self.device)
        img = to_device(batch["image"], self.device)
        toks = self.clip_tokenize(batch["question"])
        B = img.shape[0]
        q = torch.empty((B, self.embed_dim), device=self.device, dtype=torch.float32)
        di = self.image_encoder.out_dim
        s_img.wait_stream(cur)
        img.record_stream(s_img)
        q.record_stream(s_img)
        with torch.cuda.stream(s_img):
            _, other_out, _ = encode_towers(
                self.image_encoder, img, CLS, out_a=q, out_a_bstride=self.embed_dim,
                vit_b=other_vit, mode_b=other_mode, text=self.text_encoder, tokens=toks,
                out_t=q[:, di:], out_t_bstride=self.embed_dim)
        other_out.record_stream(cur)
        self._pending_img = (batch["image"], q, tuple(batch["question"]))
        return other_out, s_img

    def _key(self, batch):
        # the batch's image tensor is kept alive by whoever holds the key, so an equal id() means
        # the same object
        return (id(batch["image"]), tuple(batch["question"]), self.retrieval_k,
                self.is_training_phase)

    def prefetch(self, batch, other_vit=None, other_mode: int = CLS, slot: int = 0):
        """Serving-loop lookahead: enqueue all of ``batch``'s device-side retrieval work — the
        query towers (in lockstep with ``other_vit`` over the same images when given, as
        ``encode_image_pair``), the index scan, and the copy of its top-k into pinned host
        memory — on the retrieval stream, and return without waiting.  The next
        ``retrieve_closest_qa_pairs(batch)`` waits for that copy only, so a caller can enqueue
        batch i+1's towers before it blocks on batch i's retrieval result.  Returns
        (``other_vit``'s output or None, an event recorded after the towers: wait on it, not on
        the stream, which by then may hold the next batch's work).  ``slot`` (0-3) runs the
        towers on that workspace slot and its own stream."""
        return self.prefetch_many([batch], other_vit, other_mode, slot)[0]

    def prefetch_many(self, batches, other_vit=None, other_mode: int = CLS, slot: int = 0):
        """``prefetch`` of 1-2 batches with ONE tower pass over all their images when they are of
        equal size (the ViTs over the images concatenated, each batch's questions as its own
        text run: every row bit-identical to the per-batch pass; unequal batches get a pass
        each) and one search per batch.  Returns a list of
        (other output or None, towers event), one per batch."""
        if self.index is None:
            raise RuntimeError("create_retrieval_dataset() / set_index() first")
        if not 1 <= len(batches) <= 2:
            raise ValueError(f"prefetch_many: {len(batches)} batches (1 or 2)")
        if len({b["image"].shape[0] for b in batches}) > 1:  # one pass needs equal batches
            return [self.prefetch_many([b], other_vit, other_mode, slot)[0] for b in batches]
        s_img = self._slot_stream(int(slot))
        cur = torch.cuda.current_stream(self.device)
        imgs = [to_device(b["image"], self.device) for b in batches]
        img = imgs[0] if len(imgs) == 1 else torch.cat(imgs)
        toks = [self.clip_tokenize(b["question"]) for b in batches]
        sizes = [x.shape[0] for x in imgs]
        rows = [sum(sizes[:j]) for j in range(len(sizes))]
        q = torch.empty((img.shape[0], self.embed_dim), device=self.device, dtype=torch.float32)
        di = self.image_encoder.out_dim
        kk = self._search_k()
        s_img.wait_stream(cur)
        img.record_stream(s_img)
        q.record_stream(s_img)
        with torch.cuda.stream(s_img):
            _, other_out, _ = encode_towers_multi(
                self.image_encoder, img, CLS, out_a=q, out_a_bstride=self.embed_dim,
                vit_b=other_vit, mode_b=other_mode, text=self.text_encoder, tokens=toks,
                out_t=[q[r:r + n, di:] for r, n in zip(rows, sizes)],
                out_t_bstride=[self.embed_dim] * len(toks), slot=int(slot))
            towers = torch.cuda.Event()
            towers.record(s_img)
        if other_out is not None:
            other_out.record_stream(cur)
        out = []
        for b, r, n in zip(batches, rows, sizes):
            qb = q[r:r + n]
            host = done = None
            if isinstance(self.index, DeviceIndex):  # a sharded search exchanges: in _topk
                s_scan = self._scan_stream()
                s_scan.wait_event(towers)
                q.record_stream(s_scan)
                with torch.cuda.stream(s_scan):
                    dist, ids = self.index.search(qb, kk)
                    both = torch.cat([ids.to(torch.float64), dist.to(torch.float64)], 1)
                    host = torch.empty(both.shape, dtype=torch.float64, pin_memory=True)
                    host.copy_(both, non_blocking=True)
                    done = torch.cuda.Event()
                    done.record(s_scan)
            while len(self._prefetched) >= 8:  # never consumed (an abandoned loop): drop oldest
                self._prefetched.pop(next(iter(self._prefetched)))
            self._prefetched[self._key(b)] = (host, done, qb, towers, kk, b["image"])
            out.append((None if other_out is None else other_out[r:r + n], towers))
        return out

    def encode_queries(self, batch) -> torch.Tensor:
        """[CLS image embedding ‖ EOT text embedding] fp32 [B, 1024] on the device
        (dataset/VQAFeatureDataset.py:189-191, 146-148): the image and text towers in one
        lockstep pass (``encoders.encode_towers``, their projections share launches) on the
        retrieval stream, writing their halves of the query rows in place; the caller's stream
        waits for it.  When ``encode_image_pair`` already encoded this batch, its rows are
        returned."""
        cur = torch.cuda.current_stream(self.device)
        s_img = self._streams()
        pending = getattr(self, "_pending_img", None)
        self._pending_img = None
        if (pending is not None and pending[0] is batch["image"]
                and pending[2] == tuple(batch["question"])):
            cur.wait_stream(s_img)
            return pending[1]
        img = to_device(batch["image"], self.device)
        toks = self.clip_tokenize(batch["question"])
        q = torch.empty((img.shape[0], self.embed_dim), device=self.device, dtype=torch.float32)
        di = self.image_encoder.out_dim
        s_img.wait_stream(cur)
        q.record_stream(s_img)
        img.record_stream(s_img)
        with torch.cuda.stream(s_img):
            encode_towers(self.image_encoder, img, CLS, out_a=q, out_a_bstride=self.embed_dim,
                          text=self.text_encoder, tokens=toks, out_t=q[:, di:],
                          out_t_bstride=self.embed_dim)
        cur.wait_stream(s_img)
        return q

    def _encode_two(self, b0, b1, slot: int = 0, join: bool = True) -> torch.Tensor:
        """encode_queries of two equal-sized batches in one tower pass: rows [b0 ; b1], on
        tower workspace ``slot`` and its stream (join=False: the caller's stream is not made to
        wait for it; the caller joins ``self._slot_stream(slot)`` itself)."""
        cur = torch.cuda.current_stream(self.device)
        s_img = self._slot_stream(slot)
        img = torch.cat([to_device(b["image"], self.device) for b in (b0, b1)])
        toks = [self.clip_tokenize(b["question"]) for b in (b0, b1)]
        n = b0["image"].shape[0]
        q = torch.empty((2 * n, self.embed_dim), device=self.device, dtype=torch.float32)
        di = self.image_encoder.out_dim
        s_img.wait_stream(cur)
        q.record_stream(s_img)
        img.record_stream(s_img)
        with torch.cuda.stream(s_img):
            encode_towers_multi(self.image_encoder, img, CLS, out_a=q,
                                out_a_bstride=self.embed_dim, text=self.text_encoder,
                                tokens=toks, out_t=[q[:n, di:], q[n:, di:]],
                                out_t_bstride=[self.embed_dim] * 2, slot=slot)
        if join:
            cur.wait_stream(s_img)
        return q

    # ---- index -------------------------------------------------------------------------------
    def set_index(self, embeddings: torch.Tensor, answers: list, question_info: dict,
                  retrieval_k: int = 15, is_training_phase: bool = False):
        self.retrieval_k = retrieval_k
        self.is_training_phase = is_training_phase
        self.retrieval_answers = list(answers)
        self.retrieval_question_info = {k: list(v) for k, v in question_info.items()}
        emb = embeddings.detach().to(torch.float32)
        if self.group is not None:
            from .distributed import ShardedIndex
            self.index = ShardedIndex(emb, self.device, self.metric, group=self.group,
                                      max_batch=self.max_batch)
        else:
            self.index = DeviceIndex(emb, self.device, self.metric)
        self.retrieval_embeddings = emb
        self._cache_key = None
        self._recent = {}

    def _cache_paths(self, root, data_loader):
        n = len(getattr(data_loader, "dataset", []))
        name = getattr(getattr(data_loader, "dataset", None), "name", "dataset")
        d = os.path.join(root, type(self).__name__, f"{name}_{n}")
        return d, os.path.join(d, "embedding.pt"), os.path.join(d, "answers.json"), \
            os.path.join(d, "question_info.json")

    @staticmethod
    def _ref_paths(d):
        """The reference's cache files (dataset/VQAFeatureDataset.py:122-124)."""
        return (os.path.join(d, "embedding.pt"), os.path.join(d, "answers.pkl"),
                os.path.join(d, "answer_types.pkl"))

    def _encode_loader(self, data_loader):
        """[img ‖ txt] rows of every batch (dataset/VQAFeatureDataset.py:145-161)."""
        embs, answers = [], []
        info = {"question_type": [], "question_id": [], "question": []}
        # query rows stay on the device until the end: the host never waits on a batch, so
        # the tower passes of consecutive batches queue back to back on the GPU; two equal-sized
        # batches share one pass (twice the GEMM rows, every row bit-identical), and consecutive
        # passes alternate between two tower workspace slots and their streams, so one pass's
        # under-filled launches (the 768-column GEMMs, attention, norms) overlap the next's
        pend = None
        npass = 0
        used = set()
        for batch in data_loader:
            answers.extend(batch["answer"])
            info["question_type"].extend(batch["question_type"])
            info["question_id"].extend(batch["question_id"])
            info["question"].extend(batch["question"])
            if pend is None:
                pend = batch
            elif pend["image"].shape[0] == batch["image"].shape[0]:
                # slots 0 and 2: a pass's two text runs use text workspaces slot and slot + 1
                slot = 2 * (npass % self.BUILD_SLOTS)
                embs.append(self._encode_two(pend, batch, slot=slot, join=False))
                used.add(slot)
                npass += 1
                pend = None
            else:
                embs.append(self.encode_queries(pend))
                pend = batch
        if pend is not None:
            embs.append(self.encode_queries(pend))
        cur = torch.cuda.current_stream(self.device)
        for slot in used:
            cur.wait_stream(self._slot_stream(slot))
        emb = (torch.cat(embs, 0) if embs else
               torch.empty((0, self.embed_dim), device=self.device)).cpu()
        return emb, answers, info

    def create_retrieval_dataset(self, data_loader, prefix=None, is_training_phase=True,
                                 retrieval_k=15, use_additional_data=False, cache_dir="cache",
                                 layout="native", cache_name=None):
        """dataset/VQAFeatureDataset.py:118-185.

        ``layout="native"`` (default): cache under a key that includes the dataset name and
        size, tensor + JSON files (the reference's class-name key collides).
        ``layout="reference"``: the reference's own files and key, ``<cache_dir>/<cache_name>/
        embedding.pt | answers.pkl | answer_types.pkl`` (read when embedding.pt and answers.pkl
        exist, as :126), so a cache the reference built is served and one built here is the
        reference's; files are read with loaders that execute nothing (``torch.load(...,
        weights_only=True)``, ``read_pickled_data``)."""
        if layout == "reference":
            d = os.path.join(cache_dir, cache_name or type(self).__name__)
            emb_p, ans_p, info_p = self._ref_paths(d)
            if os.path.exists(emb_p) and os.path.exists(ans_p):
                emb = torch.load(emb_p, map_location="cpu", weights_only=True).float()
                answers = read_pickled_data(ans_p)
                info = read_pickled_data(info_p) if os.path.exists(info_p) else {}
            else:
                emb, answers, info = self._encode_loader(data_loader)
                os.makedirs(d, exist_ok=True)
                torch.save(emb, emb_p)
                with open(ans_p, "wb") as f:
                    pickle.dump(answers, f)
                with open(info_p, "wb") as f:
                    pickle.dump(info, f)
        elif layout == "native":
            d, emb_p, ans_p, info_p = self._cache_paths(cache_dir, data_loader)
            if os.path.exists(emb_p) and os.path.exists(ans_p) and os.path.exists(info_p):
                emb = torch.load(emb_p, map_location="cpu", weights_only=True).float()
                with open(ans_p) as f:
                    answers = json.load(f)
                with open(info_p) as f:
                    info = json.load(f)
            else:
                emb, answers, info = self._encode_loader(data_loader)
                os.makedirs(d, exist_ok=True)
                torch.save(emb, emb_p)
                with open(ans_p, "w") as f:
                    json.dump(answers, f)
                with open(info_p, "w") as f:
                    json.dump(info, f)
        else:
            raise ValueError(f"layout {layout!r} (native or reference)")
        if use_additional_data:
            # :169-181 (ROCO synthetic corpus); question-info dicts are merged key by key where
            # the reference calls .extend on a dict (F9)
            extra = os.path.join("synthetic_data", "cache", "ROCOFeatureDataset")
            emb = torch.cat([emb, torch.load(os.path.join(extra, "embedding.pt"),
                                             map_location="cpu", weights_only=True).float()], 0)
            if layout == "reference":
                _, e_ans, e_info = self._ref_paths(extra)
                more_ans, more = read_pickled_data(e_ans), read_pickled_data(e_info)
            else:
                with open(os.path.join(extra, "answers.json")) as f:
                    more_ans = json.load(f)
                with open(os.path.join(extra, "question_info.json")) as f:
                    more = json.load(f)
            answers = list(answers) + list(more_ans)
            info = {k: list(info.get(k, [])) + list(more.get(k, [])) for k in set(info) | set(more)}
        self.set_index(emb, answers, info, retrieval_k, is_training_phase)

    # ---- search --------------------------------------------------------------------------------
    def _topk(self, batch):
        """(dists [B, s+k], ids [B, s+k]) as host numpy, s = 1 in the training phase.  Cached
        while the same batch object (same images, same questions) is queried again."""
        key = self._key(batch)
        if self.cache_enabled and key == self._cache_key:
            return self._cache_val
        if self.cache_enabled:  # a batch searched a few batches ago (a serving loop ran ahead)
            ent = self._recent.get(key)
            if ent is not None and ent[1] is batch["image"]:
                return ent[0]
        if self.index is None:
            raise RuntimeError("create_retrieval_dataset() / set_index() first")
        kk = self._search_k()
        pre = self._prefetched.pop(key, None)
        if pre is not None and pre[0] is not None:  # prefetch(): scan + copy already enqueued
            pre[1].synchronize()
            both = pre[0].numpy()
        else:
            if pre is not None:  # towers enqueued by prefetch(), the (sharded) search here
                q = pre[2]
                torch.cuda.current_stream(self.device).wait_event(pre[3])
            else:
                q = self.encode_queries(batch)
            dist, ids = self.index.search(q, kk)
            both = torch.cat([ids.to(torch.float64), dist.to(torch.float64)], 1).cpu().numpy()
        val = (both[:, kk:].astype(np.float32), both[:, :kk].astype(np.int64))
        self._cache_key, self._cache_val, self._cache_ref = key, val, batch["image"]
        self._recent[key] = (val, batch["image"])
        while len(self._recent) > self.RECENT:
            self._recent.pop(next(iter(self._recent)))
        return val

    def _search_k(self) -> int:
        """Columns of the search: retrieval_k (+ the skipped self-match in the training phase),
        at most the index rows — the reference slices argsort(...)[:, s:s + retrieval_k] out of
        a full sort, which holds only N columns (dataset/VQAFeatureDataset.py:194-197)."""
        kk = self.retrieval_k + (1 if self.is_training_phase else 0)
        answers = getattr(self, "retrieval_answers", None)
        n = len(answers) if answers else kk
        return max(1, min(kk, n))

    def retrieve_closest_qa_pairs(self, batch, return_ans=False, return_info=None,
                                  return_dists=False, use_quantifier=True):
        """dataset/VQAFeatureDataset.py:187-246."""
        dists, ids = self._topk(batch)
        s = 1 if self.is_training_phase else 0
        sel = ids[:, s:s + self.retrieval_k]
        answers = [[self.retrieval_answers[j] for j in row] for row in sel]
        if return_ans:
            return answers
        if return_info:
            out = []
            for row in sel:
                info = []
                for j in row:
                    info.extend(self.retrieval_question_info[e][j] for e in return_info)
                out.append(info)
            return out
        if return_dists:
            return list(zip(answers, dists[:, 0:self.retrieval_k]))
        return [vote_prompt(r, use_quantifier) for r in answers]
