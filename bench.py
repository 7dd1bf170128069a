"""bench.py — QA pairs/s of the encode -> retrieve -> prompt -> T5-generate hot path on MI355X.

Metric (BASELINE.json): "QA pairs/sec (encode+retrieve+T5 gen), SLAKE k=1; 1/2/4/8 GPU scaling".
Workload (config C2): per GPU a batch of B=16 QA pairs (synthetic 224x224
images in pageable host memory, copied to the device inside the step as main.py's DataLoader
batches are, + new random-word questions every step), clip.tokenize (byte-level BPE) on the
host, retrieval over a 6,500 x 1,024 fp32 index (k=1, test phase), prompt build + SentencePiece
T5 tokenisation on the host, ViT-B/32 token features, t5-small encoder and 20 forced greedy
decode steps, answers decoded on the host.  One step =
``T5VisionModel.predict(batch)`` with ``VQARetrieval.retrieve_closest_qa_pairs`` as the
retrieval function (the reference's main.py --test inner loop, main.py:262-263), i.e. every
stage of the path, host included.  Weights are seeded random (no checkpoints offline).

N > 1: one process per GPU (torch.distributed.run), each with its own batch of 16 (weak
scaling); C2's 26.6 MB index is replicated per rank (no data-path collective; --index-sharding
shard row-shards it with one exchange per batch).  The ``c5_scan`` line is the row-sharded 1M x
512 search (strong scaling, one all_gather of per-shard top-k); its ``end_to_end_t5_base`` entry
is config C5 end to end over the rows/N shards (weak: 256 questions per GPU per batch).

Prints ONE JSON line (rank 0).  ``roofline`` is for the dominant kernel (the split-bf16 MFMA
GEMM, fp32-accurate): the launches of a pass over the same steps are recorded and replayed back
to back with one hipEvent pair around the replay (its ``in_serving_loop`` entry times the same
launches inside the pipeline, sharing the chip with the decodes); ``traffic`` comes from the
committed rocprofv3 PMC summary of this command (profiles/*pmc_gemm.json).  ``cpu_baseline`` is the CPU oracle
pipeline (torch-CPU fp32, KV-cached greedy decode) on a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from multimodalpromptretrieval_amd import _lib  # noqa: E402
from multimodalpromptretrieval_amd import synthetic as syn  # noqa: E402
from multimodalpromptretrieval_amd import serving  # noqa: E402
from multimodalpromptretrieval_amd.serving import lookahead, pipelined  # noqa: E402
from multimodalpromptretrieval_amd.tokenization import SpmT5Tokenizer, clip_tokenize  # noqa: E402

CONFIGS = {
    # name: (batch per GPU, index rows, index dim, k, t5 config)
    "c2": dict(B=16, N=6500, D=1024, k=1, t5="t5-small",
               desc="SLAKE k=1: ~6.5k x 1024 index, t5-small + ViT-B/32, batch 16"),
    "c3": dict(B=16, N=10000, D=1024, k=3, t5="t5-small",
               desc="VQA_RAD->SLAKE k=3: 10k x 1024 combined index, batch 16"),
    "c4": dict(B=16, N=65536, D=1024, k=5, t5="t5-small",
               desc="ROCO synthetic corpus k=5: 65,536 x 1024 index, batch 16"),
}
WORDS = ("what is the organ shown in this image does picture contain lung liver brain which "
         "modality used where mass abnormal left right heart kidney chest abdomen ct mri "
         "x-ray largest normal").split()
TASKS = ["organ", "modality", "position", "abnormality", "plane", "quantity", "color", "size"]
FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32, dense
BF16_MFMA_PEAK_TFLOPS = 2516.8  # MI355X_MICROARCH.md: bf16 dense = 16 x the f32 MFMA rate
HBM_PEAK_GBS = 8000.0


def _pmc_traffic():
    """HBM bytes per GEMM launch from the committed rocprofv3 PMC summary of this command
    (tools/pmc_traffic.py: FETCH_SIZE x 2 (gfx950 half-count of wide streaming reads) +
    WRITE_SIZE, separate --pmc passes, windowed to the replay).  (bytes, source) or (None, None)."""
    import glob
    import re

    def _version(path):  # r<round>_v<n>_pmc_gemm.json, newest last (mtimes do not survive a checkout)
        m = re.search(r"r(\d+)_v(\d+)_pmc_gemm\.json$", path)
        return (int(m.group(1)), int(m.group(2))) if m else (-1, -1)
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_gemm.json")), key=_version)
    if not files:
        return None, None
    with open(files[-1]) as f:
        j = json.load(f)
    return j.get("traffic_bytes_per_launch"), os.path.relpath(files[-1], ROOT)


C5 = dict(N=1 << 20, D=512, B=256, k=5)


def c5_scan(world, rank, device, group, rdev, iters=20):
    """Config C5's retrieval core: a 1,048,576 x 512 fp32 index row-sharded
    over the ranks (rows/W each, built on device from chunk-seeded streams, so the global index
    is the same at every W), one batch of 256 queries held by every rank, k = 5.  One search =
    ShardedIndex.search_all: the local large-batch scan of the rank's shard (coarse bf16 scan +
    exact re-rank), ONE all_gather of the per-shard top-k (north_star: RCCL all-gather over
    xGMI), merge.  Strong scaling (fixed index and query batch); the ids checksum is identical at
    every W."""
    from multimodalpromptretrieval_amd.distributed import ShardedIndex, shard_bounds
    from multimodalpromptretrieval_amd.index import DeviceIndex
    n, d, B, k = C5["N"], C5["D"], C5["B"], C5["k"]
    lo, hi = shard_bounds(n, world, rank)
    rows = syn.index_rows_device(7, lo, hi, d, device)
    gq = torch.Generator(device=device).manual_seed(8)
    q_all = torch.randn((B, d), device=device, generator=gq) * 0.3
    q = q_all
    six = ix = None
    if world > 1:
        six = ShardedIndex(rows, device, group=group, rows_are_local=True, row_offset=lo)
        search = six.search_all
    else:
        ix = DeviceIndex(rows, device)
        search = ix.search
    del rows
    for _ in range(3):
        search(q, k)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        dist_k, ids = search(q, k)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    chk = torch.tensor([float(ids.sum())], device=rdev, dtype=torch.float64)
    if world > 1:
        t = torch.tensor([el], device=rdev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        dist.all_reduce(chk, op=dist.ReduceOp.MAX)  # every rank holds the whole result
    ms = el / iters * 1e3
    tf = 2.0 * n * d * B / (ms * 1e-3) / 1e12
    search = six = ix = None
    torch.cuda.empty_cache()
    # the coarse path's algorithmic bytes: the bf16 index copy read once per search (2 B per
    # element), against the whole search's time at this rank count (every rank's shard in
    # parallel): a lower bound on the coarse kernel's own fraction
    gbs = n * d * 2 / (ms * 1e-3) / 1e9
    return {"workload": "C5: 1,048,576 x 512 fp32 index, rows/W per rank; 256 queries on every "
                        "rank, k=5, one all_gather of per-shard top-k",
            "ms_per_search": round(ms, 3), "queries_per_s": round(B / (ms * 1e-3), 1),
            "scan_tflops_aggregate": round(tf, 2), "scaling": "strong",
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS * world,
                         "unit": "GB/s", "frac": round(gbs / (HBM_PEAK_GBS * world), 4),
                         "note": "bf16 index bytes (N x D x 2, read once per search by the "
                                 "register-query coarse kernel) / the whole search time (coarse "
                                 "scan, select + exact re-rank, gated fallback launches, merge, "
                                 "all_gather at W > 1) against W x 8 TB/s"},
            "ids_checksum": int(chk.item())}


N_IMAGES = 8  # distinct host image tensors cycled by the batches (every batch's questions differ)


# RCCL all_gather over xGMI, modelled (one GPU per box here: an N-rank RCCL run is not
# available to this build; the driver's 8-GPU runs measure it): alpha + bytes / beta
AG_ALPHA_US = 20.0
AG_BETA_GBS = 50.0


def _projected_shard_class():
    from multimodalpromptretrieval_amd.distributed import ShardedIndex

    class ProjectedShard(ShardedIndex):
        """One rank's shard of a W-rank row-sharded index, run on a world-1 RCCL group: the
        product's ShardedIndex (local scan, pack, all_gather, merge) whose all_gather fills
        block 0 of a [W, B, k] receive buffer whose other W - 1 blocks hold this shard's first
        top-k again with ids offset by the shard size and distances set to +inf (written once,
        untimed), so the merge reads and orders W x k candidates per query as rank r of W does
        and returns this shard's own top-k.  Two receive buffers alternate (two
        batches are in flight).  Used by the one-GPU strong-scaling projection only."""

        def __init__(self, rows, device, virtual_world: int, group=None):
            super().__init__(rows, device, group=group, rows_are_local=True, row_offset=0)
            self.virtual_world = int(virtual_world)
            self._recv = []
            self._calls = 0

        def _buffers(self, packed):
            W, B = self.virtual_world, packed.shape[0]
            if not self._recv or self._recv[0].shape[0] != W * B:
                rest = packed.repeat(W, 1, 1)
                offs = (torch.arange(W, device=packed.device, dtype=torch.float64)
                        .repeat_interleave(B) * self.n_local)
                rest[..., 1] += offs[:, None]
                # the stand-in shards' candidates rank behind this shard's (+inf distances):
                # the merge still reads and orders all W x k of them, and its result is this
                # shard's own top-k (copies at equal distances would win ties by fill order)
                rest[B:, :, 0] = float("inf")
                self._recv = [rest, rest.clone()]
                torch.cuda.current_stream(packed.device).synchronize()
            recv = self._recv[self._calls % 2]
            self._calls += 1
            return recv

        def _recv_blocks(self, q, B: int, k: int):  # the native path (mpr_sharded_search_all)
            if self.virtual_world == 1:
                return super()._recv_blocks(q, B, k)
            if not self._recv:
                self._buffers(self._pack(*self._local.search(q, k)))
                self._calls = 0
            return self._buffers(self._recv[0][:B]), self.virtual_world

        def _gather(self, packed, async_op: bool = False):  # the Python path
            if self.virtual_world == 1:
                return super()._gather(packed, async_op)
            recv = self._buffers(packed)
            work = dist.all_gather_into_tensor(recv[:packed.shape[0]], packed, group=self.group,
                                               async_op=async_op)
            return recv, work

    return ProjectedShard


def _world1_group(device):
    """A one-rank RCCL process group on this GPU (the projection's collectives are then real
    RCCL calls).  Returns (group, created)."""
    if dist.is_initialized():
        return dist.group.WORLD, False
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0,
                            world_size=1, device_id=device)
    return dist.group.WORLD, True


def c5_projection(device, iters: int = 20):
    """Config C5's strong scaling, projected from one GPU: the exact per-rank
    work of W = 2, 4, 8 — the search of a 1,048,576 / W-row shard for all 256 queries (k = 5)
    and the merge of the W x 5 gathered candidates per query — timed here, plus a modelled RCCL
    all_gather of the W x 256 x 5 packed (dist, id) float64 pairs.  The pipelined form runs the
    product's ShardedIndex.search_all_many on a world-1 RCCL group (ProjectedShard: the merge
    reads W x k candidates), timed with hipEvents on the caller's stream."""
    from multimodalpromptretrieval_amd.index import DeviceIndex, topk_merge
    n, d, B, k = C5["N"], C5["D"], C5["B"], C5["k"]
    gq = torch.Generator(device=device).manual_seed(8)
    q = torch.randn((B, d), device=device, generator=gq) * 0.3
    group, created = _world1_group(device)
    ProjectedShard = _projected_shard_class()

    def timed_sharded(six):
        """Per-batch time of ShardedIndex.search_all_many over `iters` batches back to back
        (two in flight on its two streams); returns (us, ids of the last batch)."""
        last = None
        for rep in range(2):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for out in six.search_all_many((q for _ in range(iters if rep else 4)), k):
                last = out
            e1.record()
            e1.synchronize()
        return e0.elapsed_time(e1) / iters * 1e3, last[1]

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / iters * 1e3  # us

    streams = [torch.cuda.Stream(device), torch.cuda.Stream(device)]

    def timed_pipelined(fn):
        """fn per batch on two streams alternately (ShardedIndex.search_all_many's two in
        flight): per-batch time of back-to-back batches, each stream's tail (re-rank, merge)
        under the other's next scan."""
        cur = torch.cuda.current_stream(device)
        for rep in range(2):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for st in streams:
                st.wait_stream(cur)
            for i in range(iters if rep else 4):
                with torch.cuda.stream(streams[i % 2]):
                    fn()
            for st in streams:
                cur.wait_stream(st)
            e1.record()
            e1.synchronize()
        return e0.elapsed_time(e1) / iters * 1e3  # us

    out = {}
    t1 = t1_tp = None
    for W in (1, 2, 4, 8):
        rows = syn.index_rows_device(7, 0, n // W, d, device)
        if W == 1:
            ix = DeviceIndex(rows, device)
            del rows
            t1 = timed(lambda: ix.search(q, k))
            t1_tp = timed_pipelined(lambda: ix.search(q, k))
            ix.close()
            ix = None
            torch.cuda.empty_cache()
            out["1"] = {"search_us": round(t1, 1), "projected_us": round(t1, 1),
                        "pipelined_us": round(t1_tp, 1)}
            continue
        six = ProjectedShard(rows, device, W, group)
        del rows
        ix = six._local
        dl, il = ix.search(q, k)
        cd = dl.repeat(1, W).contiguous()
        ci = (il.repeat(1, W) + torch.arange(W, device=device).repeat_interleave(k)
              * (n // W)).contiguous()
        # the merge's cost on the GPU timeline: search + merge back to back minus the search (a
        # merge timed alone is a host-bound Python call, ~11 us against a ~4 us kernel)
        t_alone = timed(lambda: topk_merge(cd, ci, k))
        # the difference of two timed loops: median over 5 alternations (one pair is +-10 us)
        diffs, searches = [], []
        for _ in range(5):
            searches.append(timed(lambda: ix.search(q, k)))
            diffs.append(timed(lambda: (ix.search(q, k), topk_merge(cd, ci, k))) - searches[-1])
        t_search = float(np.median(searches))
        t_merge = max(0.0, float(np.median(diffs)))
        # the product's pipelined sharded search (search_all_many on the RCCL group)
        t_tp, ids_tp = timed_sharded(six)
        same = bool(torch.equal(ids_tp, il))
        six = ix = None
        torch.cuda.empty_cache()
        ag_bytes = W * B * k * 16
        t_ag = AG_ALPHA_US + ag_bytes / (AG_BETA_GBS * 1e3)
        tot = t_search + t_merge + t_ag
        tot_tp = max(t_tp, t_ag)
        out[str(W)] = {"search_us": round(t_search, 1), "merge_us": round(t_merge, 1),
                       "merge_us_alone": round(t_alone, 1),
                       "all_gather_us_model": round(t_ag, 1), "projected_us": round(tot, 1),
                       "speedup": round(t1 / tot, 2),
                       "pipelined_us": round(t_tp, 1),
                       "pipelined_projected_us": round(tot_tp, 1),
                       "pipelined_speedup": round(t1_tp / tot_tp, 2),
                       "pipelined_ids_equal_search": same}
    if created:
        dist.destroy_process_group()
    out["model"] = (f"per rank: the W-shard search (timed) + merge of W x {k} candidates (timed behind the "
                    f"search: the marginal GPU-timeline cost) + "
                    f"all_gather {AG_ALPHA_US} us + bytes / {AG_BETA_GBS} GB/s (modelled); "
                    f"pipelined: ShardedIndex.search_all_many itself on a world-1 RCCL group "
                    f"(two batches in flight on its two streams, each one mpr_sharded_search_all "
                    f"call: local scan, pack, the merge of W x {k} candidates per query; at one "
                    f"rank there is no collective to make), per batch max(that measured time, "
                    f"the all_gather model), against the one-GPU DeviceIndex.search on two "
                    f"alternating streams")
    return out


def c4_projection(device, iters: int = 50):
    """Config C4's retrieval at W = 1, 2, 4, 8 GPUs, projected from one GPU (SURVEY.md §8(e),
    BASELINE config 4: a 65,536 x 1,024 index row-sharded over the ranks, 16 questions per rank
    per step, k = 5).  Per rank per step, ShardedIndex.search does: an all_gather of the ranks'
    16-query blocks, the local scan of all 16 W queries over the 65,536 / W-row shard, an
    all_to_all of the [16 W, 5] candidates back to their owners, and the merge of W x 5
    candidates for its own 16 queries.  The scan and the merge are timed here on the exact
    per-rank shapes (hipEvents, back to back); the two collectives are modelled (alpha + bytes /
    beta each, as the C5 projection's all_gather).  Weak scaling: every rank serves its own 16
    questions, so the aggregate rate is W x 16 / (per-rank time)."""
    from multimodalpromptretrieval_amd.index import DeviceIndex, topk_merge
    n, d, b, k = 65536, 1024, 16, 5

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / iters * 1e3  # us

    out = {}
    base = None
    for W in (1, 2, 4, 8):
        rows = syn.index_rows_device(11, 0, n // W, d, device)
        ix = DeviceIndex(rows, device)
        del rows
        g = torch.Generator(device=device).manual_seed(12)
        q = torch.randn((b * W, d), device=device, generator=g) * 0.3
        t_scan = timed(lambda: ix.search(q, k))
        ent = {"shard_rows": n // W, "queries_scanned": b * W, "search_us": round(t_scan, 1)}
        tot = t_scan
        if W > 1:
            dl, il = ix.search(q[:b], k)
            cd, ci = dl.repeat(1, W).contiguous(), il.repeat(1, W).contiguous()
            t_both = timed(lambda: (ix.search(q, k), topk_merge(cd, ci, k)))
            t_merge = max(0.0, t_both - t_scan)
            ag = AG_ALPHA_US + W * (b + 1) * d * 4 / (AG_BETA_GBS * 1e3)
            a2a = AG_ALPHA_US + W * b * k * 16 / (AG_BETA_GBS * 1e3)
            tot = t_scan + t_merge + ag + a2a
            ent.update({"merge_us": round(t_merge, 1), "all_gather_queries_us_model": round(ag, 1),
                        "all_to_all_us_model": round(a2a, 1)})
        ix.close()
        ix = None
        torch.cuda.empty_cache()
        base = base or tot
        ent.update({"per_rank_us": round(tot, 1),
                    "retrieval_qa_pairs_per_s": round(W * b / (tot * 1e-6), 1),
                    "aggregate_vs_1": round(W * base / tot, 2)})
        out[str(W)] = ent
    out["model"] = (f"per rank per step: the 65,536/W-row scan of 16 W queries + the merge of "
                    f"W x {k} candidates (timed, the merge as its marginal GPU-timeline cost) + "
                    f"all_gather of the query blocks + all_to_all of the candidates, each "
                    f"{AG_ALPHA_US} us + bytes / {AG_BETA_GBS} GB/s (modelled); weak scaling "
                    f"(16 questions per rank)")
    return out


class _C5Retrieval:
    """Config C5's retrieval for the end-to-end leg: the questions' CLIP text embeddings (512-d,
    the index's width) searched over the 1,048,576 x 512 index (k = 5), then the reference's
    vote / bucket prompt (dataset/VQAFeatureDataset.py:190-246 with a text-only query: the
    reference's [img || txt] rows are 1024-d, C5's index is 512-d as stated)."""

    def __init__(self, text, index, answers, k):
        self.text, self.index, self.answers, self.k = text, index, answers, k
        self._ahead = {}
        self._stream = None

    def prefetch_many(self, batches, other_vit=None, other_mode=None, slot: int = 0):
        """The serving loop's lookahead (T5VisionModel._prefetch, as VQARetrieval.prefetch_many):
        each batch's text tower, search and pinned top-k copy enqueued now on a side stream, so
        the host never waits for a search queued behind the decodes.  A row-sharded index
        exchanges candidates with the other ranks inside its search: that one stays in order."""
        from multimodalpromptretrieval_amd.index import DeviceIndex
        if not isinstance(self.index, DeviceIndex):
            return [None] * len(batches)
        dev = self.index.device
        if self._stream is None:
            self._stream = torch.cuda.Stream(dev)
        self._stream.wait_stream(torch.cuda.current_stream(dev))
        out = []
        for b in batches:
            toks = clip_tokenize(b["question"])
            with torch.cuda.stream(self._stream):
                q = self.text(toks)
                _, ids = self.index.search(q, self.k)
                host = torch.empty(ids.shape, dtype=ids.dtype, pin_memory=True)
                host.copy_(ids, non_blocking=True)
                done = torch.cuda.Event()
                done.record(self._stream)
            while len(self._ahead) >= 8:  # never consumed: drop the oldest
                self._ahead.pop(next(iter(self._ahead)))
            self._ahead[(id(b["image"]), tuple(b["question"]))] = (host, done, b["image"])
            out.append((None, done))
        return out

    def __call__(self, batch, use_quantifier=True, **kw):
        from multimodalpromptretrieval_amd.dataset import vote_prompt
        ent = self._ahead.pop((id(batch["image"]), tuple(batch["question"])), None)
        if ent is not None and ent[2] is batch["image"]:
            ent[1].synchronize()
            rows = ent[0].tolist()
        else:
            q = self.text(clip_tokenize(batch["question"]))
            _, ids = self.index.search(q, self.k)
            rows = ids.cpu().tolist()
        return [vote_prompt([self.answers[int(j) % len(self.answers)] for j in row],
                            use_quantifier) for row in rows]


def c5_serving(world, rank, device, group, rdev, batches: int = 4):
    """Config C5 end to end: per batch of 256 questions, CLIP text tower ->
    1M x 512 search (k = 5) -> prompts -> t5-base encoder + 20 greedy steps with
    use_image_info=0 (t5-base cannot take the 512-d image tokens), through
    T5VisionModel.predict (architectures/T5VisionModel.py:196-216).  Forced 20 steps (the
    synthetic weights rarely stop).  N > 1: the index is row-sharded (rows/W per rank,
    distributed.ShardedIndex with fixed 256-query blocks: all_gather of the ranks' query blocks,
    the local scan of all W x 256, all_to_all of the candidates, merge) and every rank serves its
    own 256-question batches (weak scaling: the per-rank scan work stays that of the whole index
    for 256 queries while each GPU holds 1/W of it)."""
    from multimodalpromptretrieval_amd.distributed import ShardedIndex, shard_bounds
    from multimodalpromptretrieval_amd.encoders import DeviceCLIPText
    from multimodalpromptretrieval_amd.index import DeviceIndex
    from multimodalpromptretrieval_amd.model import T5VisionModel
    n, d, B, k = C5["N"], C5["D"], C5["B"], C5["k"]
    lo, hi = shard_bounds(n, world, rank)
    rows = syn.index_rows_device(7, lo, hi, d, device)
    if world > 1:
        ix = ShardedIndex(rows, device, group=group, rows_are_local=True, row_offset=lo,
                          max_batch=B)
    else:
        ix = DeviceIndex(rows, device)
    del rows
    text = DeviceCLIPText(syn.clip_state_dict(1), device)
    retr = _C5Retrieval(text, ix, syn.answers(n, 50), k)
    m = T5VisionModel(device, T5_version="t5-base", use_image_info=False,
                      clip_state_dict=syn.clip_state_dict(2),
                      t5_state_dict=syn.t5_state_dict(5, syn.T5_BASE),
                      tokenizer=SpmT5Tokenizer(), retrieval_function=retr).eval()
    pool = make_batches(batches + 1, B, seed=500 + rank, n_images=1)

    def timed(fn):
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], device=rdev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el, out

    os.environ["MPR_EOS_STOP_CHUNK"] = "0"  # forced 20 steps
    try:
        with torch.no_grad():
            # untimed: one predict() per batch, so every source-length bucket the timed batches
            # use has its encoder / decode graphs captured (as in a serving process past its
            # first requests); the timed calls recompute everything
            want = [m.predict(b) for b in pool]
            list(m.predict_many(pool[:2], eos_stop=False))
            # synchronous: one predict() after another (the host's text / search / prompt /
            # tokenize work of a batch leaves the GPU idle)
            el_sync, got_sync = timed(lambda: [m.predict(b) for b in pool[1:]])
            # the serving loop (T5VisionModel.predict_many): batch i+1's CLIP text, search,
            # prompts and tokenization run on the host and the prep stream while batch i's
            # 256-row decode runs on its own stream
            el, got = timed(lambda: list(m.predict_many(pool[1:], eos_stop=False)))
    finally:
        os.environ.pop("MPR_EOS_STOP_CHUNK", None)
    m = ix = text = retr = None
    torch.cuda.empty_cache()
    nb = len(pool) - 1
    return {"workload": f"C5 end to end, {world} GPU(s): 256 questions per batch per GPU -> CLIP "
                        f"text (512-d) -> 1M x 512 search k=5 (index rows/{world} per GPU) -> "
                        "prompts -> t5-base (use_image_info=0) encoder + 20 greedy steps "
                        "(T5VisionModel.predict_many: the serving loop)",
            "scaling": "weak" if world > 1 else None,
            "ms_per_batch": round(el / nb * 1e3, 2),
            "qa_pairs_per_s": round(world * nb * B / el, 1),
            "sync_ms_per_batch": round(el_sync / nb * 1e3, 2),
            "sync_qa_pairs_per_s": round(world * nb * B / el_sync, 1),
            "answers_equal_predict": bool(got == want[1:] and got_sync == want[1:])}


def make_batches(n_batches: int, B: int, seed: int, n_images: int = N_IMAGES):
    """Batches as main.py's DataLoader yields them (main.py:94-96, no pin_memory): images fp32
    [B, 3, 224, 224] in pageable HOST memory (copied to the device inside every step, as
    dataset/VQAFeatureDataset.py:189 / architectures/T5VisionModel.py:156 do), and questions
    that differ in every batch (the host tokenizers see new text every step)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    imgs = [syn.images(seed * 1000 + i, B) for i in range(min(n_images, n_batches))]
    out = []
    for i in range(n_batches):
        qs = []
        for _ in range(B):
            words = list(rng.choice(WORDS, size=int(rng.integers(6, 20))))
            words[0] = words[0].capitalize()
            qs.append(" ".join(words) + "?")
        out.append({
            # a view per batch: its own tensor object (batch identity), shared host storage
            "image": imgs[i % len(imgs)].view_as(imgs[i % len(imgs)]),
            "question": qs,
            "task": [TASKS[int(t)] for t in rng.integers(0, len(TASKS), size=B)],
            "answer": ["yes"] * B,
            "question_id": [str(i * B + j) for j in range(B)],
            "question_type": ["open"] * B,
        })
    return out


def build(cfg, device, group):
    from multimodalpromptretrieval_amd.dataset import VQARetrieval
    from multimodalpromptretrieval_amd.model import T5VisionModel
    retr_sd = syn.clip_state_dict(1)                 # vanilla CLIP (retrieval, encode_image/text)
    tok_sd = syn.clip_state_dict(2)                  # PubMedCLIP stand-in (token features)
    t5_sd = syn.t5_state_dict(3, syn.T5Config() if cfg["t5"] == "t5-small" else syn.T5_BASE)
    retr = VQARetrieval(device, clip_state_dict=retr_sd, clip_tokenizer=clip_tokenize,
                        group=group, max_batch=cfg["B"])
    X = syn.index_rows(4, cfg["N"], cfg["D"])
    info = {"question_id": [str(j) for j in range(cfg["N"])],
            "question_type": ["open"] * cfg["N"], "question": [""] * cfg["N"]}
    retr.set_index(X, syn.answers(cfg["N"], 50), info, cfg["k"], is_training_phase=False)
    retr.cache_enabled = False                        # every step re-encodes and re-scans
    model = T5VisionModel(device, clip_state_dict=tok_sd, t5_state_dict=t5_sd,
                          tokenizer=SpmT5Tokenizer(),
                          retrieval_function=retr.retrieve_closest_qa_pairs)
    model.eval()
    return model, retr, (retr_sd, tok_sd, t5_sd, X, info)


def decode_chain(model, batch, steps: int = 20, iters: int = 10):
    """The greedy decode of one 16-row batch (architectures/T5VisionModel.py:200-205), timed on
    its own with hipEvents: generate (encoder + cross K/V + 20 steps, graph replays) minus the same
    call with 0 steps.  Its roofline: every step streams the decoder's weights and the tied
    lm_head once (fp32), so bytes/step = 4 (Ld (6 d inner + 2 d dff) + V d)."""
    dev = model._device_t5()
    with torch.no_grad():
        emb, mask, _ = model.prepare_input(batch)

    def timed(n):
        dev.generate_padded(emb, mask, n)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(iters):
            dev.generate_padded(emb, mask, n)
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / iters

    # best of 3 for each: one stray host stall inside a 10-call window otherwise lands in one
    # of the two numbers and skews the difference
    full = min(timed(steps) for _ in range(3))
    enc = min(timed(0) for _ in range(3))
    dec_ms = full - enc
    rows = int(emb.shape[0])
    # t5.hip fold_rows: the folded chain below d = 768 at every row count (the env switches are
    # the A/B overrides)
    fe = os.environ.get("MPR_DECODE_FOLD")
    fold = ((fe != "0") if fe is not None else dev.d_model < 768) and \
        rows <= int(os.environ.get("MPR_DECODE_FOLD_ROWS", str(1 << 30)))
    launches = dev.n_dec * (6 if fold else 8) + 2
    d, inner, dff, V = dev.d_model, dev.inner, dev.d_ff, dev.vocab
    per_step = 4.0 * (dev.n_dec * (6 * d * inner + 2 * d * dff) + V * d)
    read = (4.0 * (dev.n_dec * (3 * d * inner + (d + inner) * (inner + d)
                                + (d + dff) * (inner + d) + d * dff) + V * d) if fold else per_step)
    gbs = per_step * steps / (dec_ms * 1e-3) / 1e9
    return {"rows": rows, "steps": steps, "ms_per_generate": round(full, 3),
            "encoder_ms": round(enc, 3), "decode_ms": round(dec_ms, 3),
            "us_per_step": round(dec_ms * 1e3 / steps, 1), "launches_per_step": launches,
            "folded_chain": fold,
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                         "algorithmic_mb_per_step": round(per_step / 1e6, 1),
                         "weight_mb_read_per_step": round(read / 1e6, 1)},
            "note": f"a chain of {launches} dependent launches per step "
                    f"({dec_ms * 1e3 / steps / launches:.1f} us each): latency-bound, not "
                    f"bandwidth-bound (DESIGN.md §3, the decode chain; folded: the decoder "
                    f"layer's two RMSNorms folded into the o / co projections)"}


def eos_leg(cfg, weights, retr, device, batches, steps: int):
    """The serving loop with greedy search's stop (architectures/T5VisionModel.py:200-205,
    GenerationMixin ends once every row emitted eos) on a T5 that answers in one token
    (synthetic.eos_early_t5; SLAKE's answers are 1-3 tokens): QA pairs/s with the stop polled
    asynchronously (mpr_t5_generate_begin / _poll) against the same model forced to 20 steps, and
    the decode steps each generate call launched."""
    from multimodalpromptretrieval_amd.model import T5VisionModel
    _, tok_sd, t5_sd, _, _ = weights
    m = T5VisionModel(device, clip_state_dict=tok_sd, t5_state_dict=syn.eos_early_t5(t5_sd),
                      tokenizer=SpmT5Tokenizer(),
                      retrieval_function=retr.retrieve_closest_qa_pairs).eval()
    out = {"model": "t5-small weights with an eos-early decoder (synthetic.eos_early_t5)"}
    with torch.no_grad():
        for stop in (False, True, False, True):  # warm, then timed
            loops = []
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in m.predict_many((batches[s % len(batches)] for s in range(steps)),
                                    eos_stop=stop, _loop_out=loops):
                pass
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            key = "eos_stop" if stop else "forced_20"
            out[key] = {"qa_pairs_per_s": round(steps * cfg["B"] / el, 1),
                        "steps_run_per_call": loops[0].steps_run}
    m = loops = None
    gc.collect()  # the eos model's device handles (held by reference cycles) go before the next leg
    torch.cuda.empty_cache()
    return out


def train_leg(cfg, weights, retr, device, batches, steps: int = 10):
    """main.py:177-188 — per step ``loss = model(batch)`` (train mode,
    dropout 0.1 at transformers' sites, training-phase retrieval that skips the self match),
    ``model.predict(batch)`` (:179), ``loss.backward()``, AdamW ``step()`` (the device handles
    predict() uses are rebuilt from the updated parameters).  ms per step, and the tiled GEMM's
    share: its algorithmic FLOPs over its own kernel time and over the step's wall time."""
    from multimodalpromptretrieval_amd.model import T5VisionModel
    _, tok_sd, t5_sd, _, _ = weights
    m = T5VisionModel(device, clip_state_dict=tok_sd, t5_state_dict=t5_sd,
                      tokenizer=SpmT5Tokenizer(), retrieval_function=retr.retrieve_closest_qa_pairs,
                      t5_dropout_rate=0.1)
    opt = torch.optim.AdamW(m.parameters(), lr=1e-5)  # main.py:149 (AdamW over parameters())
    phase = retr.is_training_phase
    retr.is_training_phase = True   # main.py:119-122: --train builds a training-phase index
    m.train()
    timings = {"forward": 0.0, "predict": 0.0, "backward_step": 0.0}

    def step(b, parts=False):
        # main.py:177-188 as written: loss.item() is the step's one read of a device value
        t0 = time.perf_counter()
        loss = m(b)
        if parts:
            torch.cuda.synchronize()
        t1 = time.perf_counter()
        m.predict(b)
        if parts:
            torch.cuda.synchronize()
        t2 = time.perf_counter()
        opt.zero_grad()
        loss.backward()
        opt.step()
        v = loss.item()
        t3 = time.perf_counter()
        if parts:
            timings["forward"] += t1 - t0
            timings["predict"] += t2 - t1
            timings["backward_step"] += t3 - t2
        return v

    try:
        # warmup through the same lookahead path as the timed steps (its hint stream, prefetch
        # slot and decode graphs are first used there; a plain-step warmup left those one-time
        # costs inside the timed window: 27-30 vs 16 ms per step)
        warm = (dict(b, image=b["image"].view_as(b["image"]))
                for b in (batches[i % len(batches)] for i in range(4)))
        for b in lookahead(warm, m):
            step(b)
        torch.cuda.synchronize()
        # main.py's training loop under the dropin launcher: the loader iterated one batch ahead
        # (serving.lookahead -> model.hint_next: the next batch's retrieval towers, scan and image
        # tokens enqueued beside this step's T5 forward / backward); every batch a new view, as
        # a DataLoader yields new tensors
        src = (dict(b, image=b["image"].view_as(b["image"]))
               for b in (batches[i % len(batches)] for i in range(steps)))
        t0 = time.perf_counter()
        losses = [step(b) for b in lookahead(src, m)]
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        # the same steps with a device sync after each part: where a step's time goes
        n_parts = max(2, steps // 2)
        for i in range(n_parts):
            step(batches[i % len(batches)], parts=True)
        # the tiled-GEMM launches of one step, recorded and replayed back to back (kernel time
        # only: mpr_probe_replay) — their algorithmic flops over that time, and that time's share
        # of the step
        torch.cuda.synchronize()
        _lib.probe_clear()
        _lib.probe_enable(3)
        step(batches[0])
        torch.cuda.synchronize()
        _lib.probe_enable(0)
        gms, gl, gflops, _ = _lib.probe_replay(1, device)
        _lib.probe_clear()
    finally:
        retr.is_training_phase = phase
    m = opt = None
    torch.cuda.empty_cache()
    ms = el / steps * 1e3
    return {"workload": f"main.py:177-188 train step: t5-small + ViT-B/32 token features, batch "
                        f"{cfg['B']}, dropout 0.1, forward + predict + backward + AdamW + "
                        f"loss.item(); the loader one batch ahead (serving.lookahead, as the "
                        f"dropin launcher iterates main.py's training loader)",
            "ms_per_step": round(ms, 2),
            "ms_per_step_parts_synced": {k: round(v / n_parts * 1e3, 2)
                                         for k, v in timings.items()},
            "qa_pairs_per_s": round(cfg["B"] / (ms * 1e-3), 1),
            "loss_first_last": [round(losses[0], 4), round(losses[-1], 4)],
            "roofline": {"bound": "mfma", "kernel": "gemm_x3_kernel (tiled split-bf16 GEMM)",
                         "gemm_launches_per_step": gl,
                         "gemm_ms_per_step": round(gms, 3),
                         "achieved": round(gflops / (gms * 1e-3) / 1e12, 2) if gms else None,
                         "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(gflops / (gms * 1e-3) / 1e12 / FP32_MFMA_PEAK_TFLOPS, 4)
                         if gms else None,
                         "gemm_share_of_wall": round(gms / ms, 4),
                         "note": "one step's tiled-GEMM launches recorded and replayed back to "
                                 "back (mpr_probe_replay): algorithmic flops / replay time; "
                                 "gemm_share_of_wall = replay time / step wall time"}}


def index_build(cfg, weights, device, n_batches: int = 48):
    """VQARetrieval.create_retrieval_dataset (dataset/VQAFeatureDataset.py
    :118-185) over a loader of synthetic batches — the retrieval ViT (CLS) + CLIP text towers per
    row, the [N, 1024] fp32 matrix written to the cache directory, the index uploaded — timed
    end to end on rank 0 (a fresh cache directory: nothing is loaded from disk)."""
    import shutil
    import tempfile
    from multimodalpromptretrieval_amd.dataset import VQARetrieval
    retr_sd = weights[0]
    r = VQARetrieval(device, clip_state_dict=retr_sd, clip_tokenizer=clip_tokenize)
    loader = make_batches(n_batches, cfg["B"], seed=7)
    out = {}
    for phase in ("warm", "timed"):
        d = tempfile.mkdtemp(prefix="mpr_ib_")
        try:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r.create_retrieval_dataset(loader, is_training_phase=False, retrieval_k=cfg["k"],
                                       cache_dir=d)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
        finally:
            shutil.rmtree(d, ignore_errors=True)
        out[phase] = el
    # the towers' GEMM flops of one build (algorithmic, from the launch probe) against the build's
    # wall time and the fp32 MFMA peak: the roofline the index build sits under
    d = tempfile.mkdtemp(prefix="mpr_ib_")
    try:
        _lib.probe_clear()
        _lib.probe_enable(1)
        r.create_retrieval_dataset(loader, is_training_phase=False, retrieval_k=cfg["k"],
                                   cache_dir=d)
        torch.cuda.synchronize()
        _lib.probe_enable(0)
        gms, gl, gflops, _ = _lib.probe_read()
        _lib.probe_clear()
    finally:
        shutil.rmtree(d, ignore_errors=True)
    rows = n_batches * cfg["B"]
    el = out["timed"]
    tf = gflops / el / 1e12
    return {"workload": f"create_retrieval_dataset over {n_batches} batches x {cfg['B']} QA "
                        f"pairs (ViT-B/32 CLS + CLIP text per row, cache write, index upload)",
            "rows": rows, "ms": round(el * 1e3, 2), "rows_per_s": round(rows / el, 1),
            "roofline": {"bound": "mfma", "gemm_gflop_per_row": round(gflops / rows / 1e9, 3),
                         "achieved": round(tf, 2), "peak": FP32_MFMA_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(tf / FP32_MFMA_PEAK_TFLOPS, 4),
                         "gemm_kernel_ms": round(gms, 2), "gemm_launches": gl,
                         "note": "GEMM algorithmic flops of the build / its wall time"}}


def pipeline_work(model, retr, batches, cfg, n: int = 16):
    """Host tokenizer cost and algorithmic FLOPs per QA pair over the first `n` timed batches.

    Host: clip.tokenize of the questions (dataset/VQAFeatureDataset.py:190), the T5 tokenizer on
    the prompts (architectures/T5VisionModel.py:161-167) and batch_decode of 20-token answers
    (:207), timed on the host alone (in the serving loop they overlap the GPU).
    FLOPs (MAC x 2, at the lengths each batch actually runs: CLIP text up to the
    batch's last EOT, the T5 source at 50 image tokens + the longest prompt): ViT-B/32 twice
    (CLS path 8.818, token path 8.856 GFLOP), CLIP text, the scan (2 N D), the t5-small encoder
    and the 20-step decode (cross K/V once, lm_head every step)."""
    dev = model._device_t5()
    sub = batches[:n]
    t_clip = t_t5 = t_dec = 0.0
    flops = 0.0
    pairs = 0
    d, dff, H, Le, Ld, V = dev.d_model, dev.d_ff, dev.num_heads, dev.n_enc, dev.n_dec, dev.vocab
    inner = dev.inner
    for b in sub:
        B = len(b["question"])
        t0 = time.perf_counter()
        toks = retr.clip_tokenize(b["question"])
        t_clip += time.perf_counter() - t0
        with torch.no_grad():
            prompts = retr.retrieve_closest_qa_pairs(b)
        sentences = [f"Answer the {t} question: " + q + p
                     for t, q, p in zip(b["task"], b["question"], prompts)]
        t0 = time.perf_counter()
        enc = model.tokenizer(sentences, padding="longest", max_length=model.max_source_length,
                              truncation=True, return_tensors="pt")
        t_t5 += time.perf_counter() - t0
        fake = torch.randint(3, 32000, (B, 21))
        fake[:, 0] = 0
        t0 = time.perf_counter()
        model.tokenizer.batch_decode(fake, skip_special_tokens=True)
        t_dec += time.perf_counter() - t0
        lt = int(toks.argmax(dim=1).max()) + 1
        L = 50 + enc["input_ids"].shape[1]
        text_mac = 12 * (lt * 512 * 1536 + 2 * 8 * lt * lt * 64 + lt * 512 * 512
                         + 2 * lt * 512 * 2048) + 512 * 512
        enc_mac = Le * ((4 * d * inner + 2 * d * dff) * L + 2 * H * 64 * L * L)
        dec_mac = Ld * 2 * d * inner * L + sum(
            Ld * (6 * d * inner + 2 * d * dff + 2 * H * 64 * (t + 1 + L)) + d * V
            for t in range(20))
        per_pair = 2 * (text_mac + enc_mac + dec_mac) + 8.818e9 + 8.856e9 + 2.0 * cfg["N"] * cfg["D"]
        flops += per_pair * B
        pairs += B
    k = 1e3 / len(sub)
    return ({"clip_tokenize": round(t_clip * k, 3), "t5_tokenize": round(t_t5 * k, 3),
             "batch_decode": round(t_dec * k, 3),
             "total": round((t_clip + t_t5 + t_dec) * k, 3)},
            flops / pairs)


def host_cpu():
    """(CPU model, physical cores of the host, CPUs this process may run on)."""
    model, cores = None, set()
    try:
        phys = None
        with open("/proc/cpuinfo") as f:
            for line in f:
                k, _, v = line.partition(":")
                k, v = k.strip(), v.strip()
                if k == "model name" and model is None:
                    model = v
                elif k == "physical id":
                    phys = v
                elif k == "core id":
                    cores.add((phys, v))
    except OSError:
        pass
    return model, len(cores) or None, len(os.sched_getaffinity(0))


def gpu_parity_outputs(model, retr, batches):
    """Per batch, what the full-size parity check compares with the CPU oracle: predict()'s
    answers, the retrieval prompts, the retrieved example ids (``return_info=["question_id"]``,
    dataset/VQAFeatureDataset.py:202-210), the ``return_dists`` values (:242-245) and the device
    query rows (to bound what the device / CPU tower difference can move)."""
    out = []
    with torch.no_grad():
        for b in batches:
            ids = [[int(s) for s in row]
                   for row in retr.retrieve_closest_qa_pairs(b, return_info=["question_id"])]
            dists = [d for _, d in retr.retrieve_closest_qa_pairs(b, return_dists=True)]
            out.append({"answers": model.predict(b), "prompts": retr.retrieve_closest_qa_pairs(b),
                        "ids": ids, "dists": dists, "query": retr.encode_queries(b).cpu()})
    return out


def cpu_baseline(cfg, weights, batches, seconds: float, gpu_out=None, serving_answers=None):
    """The CPU oracle pipeline (restated reference path, torch-CPU fp32) on a bounded sample of
    the bench's own batches.  With ``gpu_out`` (``gpu_parity_outputs`` on the same batches and
    weights) the CPU leg doubles as a full-size C2 parity check (``parity``): retrieved ids,
    distances, prompts and predict()'s answers; ``serving_answers`` are the answers the timed
    serving loop itself produced for the same batches."""
    from oracle import pipeline
    from oracle import retrieval as oret
    retr_sd, tok_sd, t5_sd, X, info = weights
    answers = syn.answers(cfg["N"], 50)
    tok = SpmT5Tokenizer()
    tok.add_tokens(["[itk]"])
    heads = 8 if cfg["t5"] == "t5-small" else 12
    cpu_batches = [{**b, "image": b["image"].cpu()} for b in batches]
    n, t0 = 0, time.perf_counter()
    cpu_out = {}
    with torch.no_grad():
        while True:
            i = n % len(cpu_batches)
            b = cpu_batches[i]
            trace = {}
            preds, prompts, _ = pipeline.predict(
                b, retr_sd, tok_sd, t5_sd, heads, X, answers, info, cfg["k"], False,
                clip_tokenize, tok, 20, forced_steps=True, trace=trace)
            cpu_out.setdefault(i, (preds, prompts, trace))
            n += 1
            el = time.perf_counter() - t0
            if el >= seconds or n >= 32:
                break
    pairs = n * cfg["B"]
    # one batch on ONE thread: the per-core rate, so the whole host's rate is bounded by
    # physical cores x that (the box's share for this GPU is 16 threads: more would take other
    # jobs' cores, so the 128-core figure is an upper bound, not a run)
    nt = torch.get_num_threads()
    torch.set_num_threads(1)
    try:
        with torch.no_grad():
            t1 = time.perf_counter()
            pipeline.predict(cpu_batches[0], retr_sd, tok_sd, t5_sd, heads, X, answers, info,
                             cfg["k"], False, clip_tokenize, tok, 20, forced_steps=True)
            one = cfg["B"] / (time.perf_counter() - t1)
    finally:
        torch.set_num_threads(nt)
    model, phys, avail = host_cpu()
    out = {"value": pairs / el, "unit": "QA pairs/s", "cores": torch.get_num_threads(),
           "kind": "port",
           "sample": f"{n} batches x {cfg['B']} QA pairs of the same workload ({el:.1f} s), "
                     f"oracle/pipeline.py (torch-CPU fp32, KV-cached greedy, 20 forced steps)",
           "cpu_model": model, "host_physical_cores": phys, "host_cpus_available": avail,
           "one_thread_value": round(one, 2),
           "whole_host_bound": round(one * phys, 1) if phys else None,
           "cores_note": "threads = this job's CPU share on the GPU box (OMP_NUM_THREADS, 16 per "
                         "GPU: the box's 8 GPUs' jobs share its physical cores, so the run stays "
                         "inside that share; SURVEY.md §8(d) asks for os.cpu_count()); "
                         "whole_host_bound = one_thread_value x physical cores, a perfect-scaling "
                         "upper bound on the whole host's CPU rate"}
    if gpu_out is not None:
        # forced steps keep finished rows on pad, as the device loop does: the decoded answers
        # compare as strings
        n_pairs = n_prompt = n_ans = n_ids = n_loop = n_loop_pred = 0
        dist_ok, margins, guards, dq, mism = True, [], [], [], []
        for i, (preds, prompts, trace) in cpu_out.items():
            g = gpu_out[i]
            n_pairs += len(preds)
            n_prompt += sum(a == b for a, b in zip(prompts, g["prompts"]))
            n_ans += sum(a == b for a, b in zip(preds, g["answers"]))
            par = oret.id_parity(g["ids"], g["dists"], g["query"], trace)
            n_ids += par["ids_equal_rows"]
            dist_ok &= par["dists_within_bound"]
            margins.append(par["min_rel_margin"])
            guards.append(par["min_margin_over_perturbation"])
            dq.append(par["max_query_delta_rel"])
            if serving_answers is not None and i < len(serving_answers):
                n_loop += sum(a == b for a, b in zip(preds, serving_answers[i]))
                n_loop_pred += sum(a == b for a, b in zip(g["answers"], serving_answers[i]))
                for r, (a, b, c) in enumerate(zip(preds, g["answers"], serving_answers[i])):
                    if not a == b == c and len(mism) < 8:
                        mism.append({"batch": i, "row": r, "oracle": a, "predict": b, "loop": c})
        out["parity"] = {
            "batches": len(cpu_out), "qa_pairs": n_pairs,
            "ids_equal": n_ids, "dists_within_bound": dist_ok,
            "prompts_equal": n_prompt, "answers_equal": n_ans,
            "serving_loop_answers_equal": n_loop if serving_answers is not None else None,
            "serving_loop_equal_predict": n_loop_pred if serving_answers is not None else None,
            "min_margin": min(margins), "min_margin_over_perturbation": min(guards),
            "max_query_delta_rel": max(dq),
            "mismatches": mism,
            "check": "CPU oracle vs the GPU on the same full-size C2 batches and weights: "
                     "retrieved example ids (return_info question_id) bit-exact per QA pair; "
                     "return_dists within the cdist bound; prompts; predict()'s greedy answers; "
                     "the answers the timed serving loop produced for these batches.  "
                     "min_margin: smallest fp64 gap between rank k and rank k+1 squared "
                     "distances / (|q|^2 + |x|^2) over the queries; "
                     "min_margin_over_perturbation: that gap / twice what the device-vs-CPU "
                     "query difference plus fp32 evaluation can move it (>= 1: equal ids are "
                     "implied by the bound)"}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=80)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-probe", action="store_true")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 sharded-scan line")
    ap.add_argument("--index-sharding", choices=["auto", "shard", "replicate"], default="auto",
                    help="N>1: row-shard the serving index over the ranks (an RCCL exchange per "
                         "batch) or keep a replica per rank; auto shards past 64 MiB (SURVEY "
                         "§8(e): C2/C3 replicas, C4's 268 MB sharded; C5's scan always sharded)")
    ap.add_argument("--no-train-leg", action="store_true",
                    help="skip the training-step line (main.py:177-188)")
    ap.add_argument("--train-leg-last", action="store_true",
                    help="time the training step after the eos-stop leg (stream-placement A/B)")
    ap.add_argument("--no-eos-leg", action="store_true",
                    help="skip the eos-stop serving line (an eos-early T5)")
    ap.add_argument("--no-index-build", action="store_true",
                    help="skip the index-build line (create_retrieval_dataset throughput)")
    ap.add_argument("--inflight", type=int, default=2,
                    help="generate calls in flight in the serving loop (predict_many; each decodes "
                         "a group of batches)")
    args = ap.parse_args()
    cfg = CONFIGS[args.config]
    # stdout carries exactly the one JSON line: everything else written to fd 1 (RCCL's version
    # banner at communicator init, library prints) goes to stderr
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch N>1 with "
                         f"torch.distributed.run --nproc-per-node {args.gpus}")
    # MPR_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs (ranks share devices round-robin,
    # collectives staged through host memory); the driver's runs use nccl (RCCL), one GPU per rank.
    backend = os.environ.get("MPR_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    device = torch.device(f"cuda:{local_rank % ndev if backend == 'gloo' else local_rank}")
    torch.cuda.set_device(device)
    group = None
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)
        group = dist.group.WORLD

    index_bytes = cfg["N"] * cfg["D"] * 4
    shard = world > 1 and (args.index_sharding == "shard" or
                           (args.index_sharding == "auto" and index_bytes > (64 << 20)))
    model, retr, weights = build(cfg, device, group if shard else None)
    # SURVEY §8(f) rank 1, measured first: a separate retrieval object on a fresh process state
    ib = None
    if rank == 0 and not args.no_index_build:
        ib = index_build(cfg, weights, device)
    # warmup batches first, then the timed steps' own: every timed step tokenizes new questions
    pool = make_batches(args.warmup + args.steps, cfg["B"], seed=100 + rank)
    warm, batches = pool[:args.warmup] or pool[:1], pool[args.warmup:]

    def barrier():
        if world > 1:
            dist.barrier()

    def main_loop(seq):
        # main.py:262-270 under the dropin launcher: predict() then the four analytics calls
        # on the retrieval dataset, per batch, the loader wrapped by serving.pipelined.  Every
        # step is a batch object of its own (a new view of the image tensor), so the retrieval's
        # per-batch search cache, on as in main.py, serves the analytics calls of that step only.
        retr.cache_enabled = True
        try:
            for b in pipelined((dict(x, image=x["image"].view_as(x["image"])) for x in seq),
                               model):
                model.predict(b)
                retr.retrieve_closest_qa_pairs(b, return_ans=True)
                retr.retrieve_closest_qa_pairs(b, return_info=["question_type"])
                retr.retrieve_closest_qa_pairs(b, return_info=["question", "question_id"])
                retr.retrieve_closest_qa_pairs(b, return_dists=True)
        finally:
            retr.cache_enabled = False

    def run(steps, pipelined=True, ahead=False, main=False, src=None, keep=None):
        # A step = one batch through encode -> retrieve -> prompt -> T5 generate.  The serving
        # loop keeps two batches in flight (T5VisionModel.predict_many): batch i+1's encoders
        # and scan run beside batch i's decode; each batch's work and answers are predict()'s.
        # Not pipelined: predict() one batch at a time (main.py:262-263), with `ahead` the
        # batches come through serving.lookahead (the dropin launcher's evaluation loop: the
        # next batch's towers and scan are enqueued before this batch's predict()).
        src = batches if src is None else src
        with torch.no_grad():
            if main:
                main_loop(src[s % len(src)] for s in range(steps))
            elif pipelined:
                # forced 20 decode steps (deterministic work per pair); `keep`
                # holds the first batches' answers (a list append: the parity check's input)
                for s, ans in enumerate(model.predict_many(
                        (src[s % len(src)] for s in range(steps)), args.inflight,
                        eos_stop=False)):
                    if keep is not None and s < 4:
                        keep.append(ans)
            else:
                seq = (src[s % len(src)] for s in range(steps))
                for b in (lookahead(seq, model) if ahead else seq):
                    model.predict(b)

    run(args.warmup, src=warm)
    # The serving loop once more, untimed, at the timed step count over the warmup batches: the
    # graphs of its decode-group shapes (rows x source-length bucket, one per generate slot) are
    # captured here, as a long-running server has them after its first groups.  At W = 5 the
    # warmup pass is one 5-batch group, so the timed run captured the 128-row and final-group
    # decode graphs itself, ~1.3 ms of host time each (MPR_GRAPH_LOG=1).
    run(args.steps, src=warm)
    run(args.warmup, pipelined=False, src=warm)
    run(args.warmup, pipelined=False, ahead=True, src=warm)
    run(args.warmup, main=True, src=warm)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    timed_answers = []
    run(args.steps, keep=timed_answers)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    rdev = device if backend == "nccl" else "cpu"
    if world > 1:
        t = torch.tensor([elapsed], device=rdev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # one-batch-at-a-time latency (predict(), nothing in flight across batches), for reference
    barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    run(args.steps, pipelined=False)
    torch.cuda.synchronize()
    sync_ms = (time.perf_counter() - t1) / args.steps * 1e3
    t1 = time.perf_counter()
    run(args.steps, pipelined=False, ahead=True)
    torch.cuda.synchronize()
    ahead_ms = (time.perf_counter() - t1) / args.steps * 1e3
    t1 = time.perf_counter()
    run(args.steps, main=True)
    torch.cuda.synchronize()
    main_ms = (time.perf_counter() - t1) / args.steps * 1e3
    # every rank (its prepare_input searches a sharded index collectively); rank 0 reports
    decode = decode_chain(model, batches[0])

    host_ms, flop_per_pair = pipeline_work(model, retr, batches, cfg)
    def train_now():
        return (train_leg(cfg, weights, retr, device, batches, steps=20)
                if rank == 0 and world == 1 and not args.no_train_leg else None)

    train = None if args.train_leg_last else train_now()
    eos = eos_leg(cfg, weights, retr, device, batches, args.steps) if not args.no_eos_leg else None
    if args.train_leg_last:  # (A/B of the stream placement: the same step after the eos leg's loops)
        train = train_now()

    roofline = None
    if not args.no_probe:
        # (1) The dominant kernel on its own: every tiled-GEMM launch of `steps` pipelined steps
        # is recorded, then re-launched back to back on this stream with one hipEvent pair
        # around the whole replay (mpr_probe_replay; two marker kernels bracket the replay so a
        # rocprofv3 trace of this same command can be windowed to it,
        # tools/prof_summary.py --replay).
        _lib.probe_clear()
        _lib.probe_enable(3)
        run(args.steps)
        torch.cuda.synchronize()
        _lib.probe_enable(0)
        ms, launches, flops, abytes = _lib.probe_replay(1, device)
        _lib.probe_clear()
        # (2) The same kernel inside the serving loop: hipEvents around each launch on its own
        # stream while the decodes of earlier batches share the chip.
        _lib.probe_enable(1)
        run(args.steps)
        torch.cuda.synchronize()
        ms_live, launches_live, flops_live, _ = _lib.probe_read()
        _lib.probe_enable(0)
        if launches:
            ach = flops / (ms * 1e-3) / 1e12
            traffic, traffic_src = _pmc_traffic()
            x3 = os.environ.get("MPR_GEMM", "") != "f32"
            roofline = {"bound": "mfma", "achieved": round(ach, 2),
                        "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": round(ach / FP32_MFMA_PEAK_TFLOPS, 4),
                        "traffic": traffic,
                        "kernel": ("gemm_x3p_kernel (the towers' GEMMs: fp32 product as 6 bf16"
                                   " v_mfma_f32_32x32x16_bf16 partial products of a 3-way bf16"
                                   " split, the fixed weights pre-split into operand order and"
                                   " loaded straight into registers; achieved/peak are fp32"
                                   " algorithmic flops against the fp32 MFMA dense peak;"
                                   " algorithmic bytes count fp32 operands)" if x3 else
                                   "gemm_f32_kernel (v_mfma_f32_32x32x2_f32 / 16x16x4)"),
                        "measured": "replay of the timed steps' launches back to back, one "
                                    "hipEvent pair around the replay",
                        "launches_per_step": round(launches / args.steps, 1),
                        "avg_launch_us": round(ms * 1e3 / launches, 2),
                        "kernel_ms_per_step": round(ms / args.steps, 3),
                        "algorithmic_gflop_per_launch": round(flops / launches / 1e9, 4),
                        "algorithmic_mb_per_launch": round(abytes / launches / 1e6, 3),
                        "traffic_source": traffic_src}
            if x3:  # what the bf16 pipe actually executes: 6 products per fp32 flop
                roofline["bf16_pipe"] = {"executed": round(6 * ach, 1),
                                         "peak": BF16_MFMA_PEAK_TFLOPS,
                                         "frac": round(6 * ach / BF16_MFMA_PEAK_TFLOPS, 4)}
            if launches_live:
                ach_live = flops_live / (ms_live * 1e-3) / 1e12
                roofline["in_serving_loop"] = {
                    "achieved": round(ach_live, 2),
                    "frac": round(ach_live / FP32_MFMA_PEAK_TFLOPS, 4),
                    "avg_launch_us": round(ms_live * 1e3 / launches_live, 2)}
        barrier()

    c5 = c4 = None
    if not args.no_c5:
        c5 = c5_scan(world, rank, device, group, rdev)
        if world == 1:
            c5["projection_1_to_8"] = c5_projection(device)
            c4 = c4_projection(device)
        c5["end_to_end_t5_base"] = c5_serving(world, rank, device, group, rdev)
        barrier()

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        gpu_out = gpu_parity_outputs(model, retr, batches[:4])
        cpu = cpu_baseline(cfg, weights, batches[:4], args.cpu_seconds, gpu_out, timed_answers)

    if rank == 0:
        pairs = world * cfg["B"] * args.steps
        value = pairs / elapsed
        line = {
            "metric": "QA pairs/sec (encode+retrieve+T5 gen), SLAKE k=1; 1/2/4/8 GPU scaling",
            "value": round(value, 2), "unit": "QA pairs/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "pipelining": f"serving loop (predict_many): next batch's towers + scan enqueued "
                          f"ahead, {serving.ServingOptions.resolve().decode_group} batches per decode "
                          f"loop, {args.inflight} generate calls in flight; ramp-up and drain "
                          f"inside the timed steps; warmup: {args.warmup} steps per leg plus one "
                          f"untimed serving-loop pass of {args.steps} steps over the warmup "
                          f"batches (decode-group graphs captured before timing)",
            "sync_ms_per_step": round(sync_ms, 3),
            "lookahead_ms_per_step": round(ahead_ms, 3),
            "main_loop_ms_per_step": round(main_ms, 3),
            "decode": decode,
            "eos_stop_leg": eos,
            "train_step": train,
            "host_tokenize_ms_per_batch": host_ms,
            "pipeline_roofline": {
                "bound": "mfma", "gflop_per_pair": round(flop_per_pair / 1e9, 3),
                "achieved": round(flop_per_pair * value / 1e12, 2),
                "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(flop_per_pair * value / 1e12 / FP32_MFMA_PEAK_TFLOPS, 4),
                "note": "algorithmic fp32 FLOPs of every stage per QA pair (two ViT-B/32, CLIP "
                        "text, scan, t5-small encoder + 20 decode steps, at each batch's run "
                        "lengths) x QA pairs/s against the fp32 MFMA dense peak"},
            "sync_note": "sync: predict() one batch at a time, nothing enqueued ahead; "
                         "lookahead: the same predict() calls with the batches iterated through "
                         "serving.lookahead (one batch ahead); main_loop: main.py's test loop "
                         "under the dropin launcher (predict() + the 4 analytics calls per batch, "
                         "the loader wrapped by serving.pipelined: a serving loop runs ahead and "
                         "predict() returns its answers, identical per batch)",
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (seeded random weights of ViT-B/32 x2, CLIP text, t5-small; "
                    "random 224x224 images in pageable host memory, copied to the device in "
                    "every step as main.py's DataLoader batches are; new random-word questions "
                    "every step through the real-algorithm tokenizers (CLIP byte-level BPE, "
                    "SentencePiece T5) on same-format stand-in vocabularies)",
            "config": {"workload": cfg["desc"], "global_batch": world * cfg["B"],
                       "index_rows": cfg["N"], "index_dim": cfg["D"], "k": cfg["k"],
                       "decode_steps": 20, "index_sharding": f"rows/{world}" if shard
                       else ("replica per rank" if world > 1 else "single"),
                       "parallelism": f"dp{world}"},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "c5_scan": c5, "c4_projection_1_to_8": c4, "index_build": ib,
        }
        print(json.dumps(line), file=json_out, flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    par = (cpu or {}).get("parity") or {}
    if par and (par["serving_loop_answers_equal"] != par["qa_pairs"] or
                par["answers_equal"] != par["qa_pairs"] or par["ids_equal"] != par["qa_pairs"]):
        # the timed loop's answers must be the reference path's (the CPU oracle's) on every
        # checked pair: a throughput from a loop that answers differently is not a result
        raise SystemExit(f"parity failure: {json.dumps(par['mismatches'])}")


if __name__ == "__main__":
    main()
