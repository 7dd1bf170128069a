"""Index sharding across the GPUs of one node.

Rank r of W holds index rows [lo_r, hi_r) (global ids preserved through ``row_offset``).  One
retrieval step per batch:
  1. all_gather of the per-rank query blocks  -> every rank scans its shard for the whole batch;
  2. local fused scan + top-k (libmpr)         -> [W*b, k] (dist, global id) candidates;
  3. all_to_all of the candidates              -> each rank receives the W shard-candidates of
                                                  its own b queries: [W, b, k];
  4. merge (libmpr topk_merge)                 -> [b, k], ties by lowest global id, so the result
                                                  is the single-GPU scan's whenever the shards'
                                                  searches take the single search's kernel path.
A row's exact fp32 distance is summed in one order per path (the exact scans' MFMA chains, the
coarse path's re-rank, scan.hip), so two rows within an ulp of each other can order differently
when a shard's size or a batch's size selects another path than the single-GPU search did:
same ids up to fp32 rounding ties (exact ties always go to the lowest id).
Messages are KB-scale (latency-bound over xGMI), so the candidates travel as ONE packed float64
tensor (ids < 2^53 and fp32 distances are exact in float64), not a collective per field.

Data-parallel ranks may hold different numbers of batches (a DataLoader sharded over ranks): a
rank that has run out calls ``finish()`` (or leaves a ``joined()`` block), which keeps answering
the other ranks' searches with empty query blocks until every rank has finished, so the
collectives stay paired and nothing deadlocks.  With ``max_batch`` set, every query block is
padded to that size and carries a header row (its real size and an active flag) through the
same all_gather: a search needs no all-reduce and no host synchronisation; without it, each
search all-reduces (MAX) the ranks' [batch size, active flag] first.

``search_all`` is the replicated-query form (every rank holds the same query batch, as in
config C5's 256-query batch): local scan of the whole batch, ONE all_gather of the per-shard
top-k (the north_star's RCCL all-gather over xGMI), and every rank merges — one collective per
search and no host synchronisation.  The collectives go through
torch.distributed (backend "nccl" = RCCL on ROCm; "gloo" in the CPU tests, which inject a CPU
searcher/merger so the sharding logic is exercised without a GPU).
"""
from __future__ import annotations

import contextlib
import os

import torch
import torch.distributed as dist

from . import _lib
from .index import L2, DeviceIndex, topk_merge


def shard_bounds(n: int, world: int, rank: int):
    per = (n + world - 1) // world
    lo = min(n, rank * per)
    return lo, min(n, lo + per)


class ShardedIndex:
    def __init__(self, rows: torch.Tensor, device, metric: int = L2, group=None,
                 rows_are_local: bool = False, row_offset: int = None, searcher=None,
                 merger=None, max_batch: int = None):
        self.group = group
        self.max_batch = int(max_batch) if max_batch else None
        self.finished = False
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.metric = metric
        self.device = torch.device(device)
        if rows_are_local:
            local, lo = rows, int(row_offset or 0)
        else:
            lo, hi = shard_bounds(rows.shape[0], self.world, self.rank)
            local = rows[lo:hi]
        if local.shape[0] < 1:
            raise ValueError(f"rank {self.rank}: empty index shard (n < world size)")
        self.n_local = local.shape[0]
        self.row_offset = lo
        self.d = rows.shape[1]
        if searcher is None:
            self._local = DeviceIndex(local, self.device, metric, row_offset=lo)
            self._search = self._local.search
        else:
            self._search = lambda q, k: searcher(local, lo, q, k)
        self._merge = merger or (lambda d, i, k: topk_merge(d, i, k, metric))
        # device kernels for the exchange's pack / merge (mpr_topk_pack / _merge_packed: no host
        # reshaping between the collective and the merge); the CPU tests inject both instead
        self._native = searcher is None and merger is None and self.device.type == "cuda"

    def _host_staged(self) -> bool:
        # gloo (CPU tests, or a one-GPU rehearsal of N ranks) moves host tensors only
        return dist.get_backend(self.group) == "gloo" and self.device.type == "cuda"

    def _reduce(self, b: int, active: int):
        """All-reduced MAX of (batch size, active flag) over the ranks (host ints)."""
        dev = "cpu" if dist.get_backend(self.group) == "gloo" else self.device
        t = torch.tensor([b, active], device=dev, dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return int(t[0]), int(t[1])

    def search(self, q: torch.Tensor, k: int):
        """q: this rank's [b, d] queries (b may differ between ranks).  Returns (dist, ids)
        [b, k].  Every rank pads its block to a common size (the group's largest b, or
        max_batch) with zero rows (their candidates are computed and dropped before the merge),
        so the collectives always see equal sizes."""
        if self.finished:
            raise RuntimeError("ShardedIndex.search after finish()")
        return self._step(q, k, active=True)[0]

    def finish(self, k: int = 1) -> int:
        """This rank has no more queries: take part in the other ranks' searches with empty
        blocks until every rank has called finish().  Returns the number of empty searches."""
        n = 0
        while True:
            _, any_active = self._step(None, k, active=False)
            if not any_active:
                break
            n += 1
        self.finished = True
        return n

    @contextlib.contextmanager
    def joined(self, k: int = 1):
        """``with index.joined(): for batch in my_batches: index.search(...)`` — finish() on
        exit, so ranks with fewer batches do not leave the others waiting."""
        try:
            yield self
        finally:
            if not self.finished:
                self.finish(k)

    def _step(self, q, k: int, active: bool):
        """One exchange round.  Returns ((dist, ids) or None, whether any rank is active)."""
        b = 0 if q is None else q.shape[0]
        fixed = self.max_batch is not None
        if fixed:
            if b > self.max_batch:
                raise ValueError(f"batch {b} > max_batch {self.max_batch}")
            bmax = self.max_batch
        else:
            bmax, any_active = self._reduce(b, int(active))
            if not any_active:
                return None, False
        qb = torch.zeros((bmax + (1 if fixed else 0), self.d), device=self.device,
                         dtype=torch.float32)
        if b:
            qb[:b] = q.to(self.device, torch.float32)
        if fixed:  # header row: [b, active]
            qb[bmax, 0] = float(b)
            qb[bmax, 1] = 1.0 if active else 0.0
        stage = self._host_staged()
        qx = qb.cpu() if stage else qb
        q_all = torch.empty((self.world * qb.shape[0], self.d), device=qx.device, dtype=qx.dtype)
        dist.all_gather_into_tensor(q_all, qx, group=self.group)
        if fixed:
            blocks = q_all.view(self.world, bmax + 1, self.d)
            if not active:  # only an idle rank reads the flags (a host sync it can afford)
                if not bool((blocks[:, bmax, 1] != 0).any()):
                    return None, False
            q_all = blocks[:, :bmax].reshape(self.world * bmax, self.d)
        q_all = q_all.to(self.device)
        d_loc, i_loc = self._padded_search(q_all, k)            # [W*bmax, k]
        packed = self._pack(d_loc, i_loc)                       # [W*bmax, k, 2] float64
        if stage:
            packed = packed.cpu()
        recv = torch.empty_like(packed)
        dist.all_to_all_single(recv, packed, group=self.group)
        if not b:
            if not active:
                return None, True
            return (torch.empty((0, k), device=self.device, dtype=torch.float32),
                    torch.empty((0, k), device=self.device, dtype=torch.int64)), True
        # [W(src shard), bmax, k] -> this rank's b real queries
        return self._merge_recv(recv.to(self.device), bmax, b, k), True

    def search_all(self, q: torch.Tensor, k: int):
        """q: the SAME [B, d] query batch on every rank (replicated).  Returns (dist, ids)
        [B, k] for the whole batch on every rank, a single-GPU search's (up to fp32 rounding ties,
        above): the local
        scan of all B queries, one all_gather of the per-shard top-k, the merge."""
        B = q.shape[0]
        q = q.to(self.device, torch.float32).contiguous()
        if self._rccl_ok(k):  # one native call: scan, pack, RCCL all_gather, merge
            return self._native_search_all(q, k)
        d_loc, i_loc = self._padded_search(q, k)                # [B, k]
        packed = self._pack(d_loc, i_loc)                        # [B, k, 2]
        stage = self._host_staged()
        if stage:
            packed = packed.cpu()
        recv, _ = self._gather(packed)
        return self._merge_recv(recv.to(self.device), B, B, k)

    def _comm(self):
        """This group's RCCL communicator (ProcessGroupNCCL._comm_ptr()) for the native sharded
        search, or 0 when there is none (gloo, CPU, an older PyTorch).  The first call makes sure
        the communicator exists (a one-element all_gather)."""
        if not hasattr(self, "_comm_cache"):
            ptr = 0
            try:
                if self._native and dist.get_backend(self.group) == "nccl":
                    x = torch.zeros(1, device=self.device)
                    dist.all_gather_into_tensor(torch.empty(self.world, device=self.device), x,
                                                group=self.group)
                    pg = self.group if self.group is not None else dist.group.WORLD
                    ptr = int(pg._get_backend(self.device)._comm_ptr())
            except (AttributeError, RuntimeError, TypeError):
                ptr = 0
            self._comm_cache = ptr
        return self._comm_cache

    def _rccl_ok(self, k: int) -> bool:
        """The native exchange applies: RCCL's symbols are loaded (another soname or an RCCL
        without them takes the torch.distributed all_gather instead) and a communicator exists."""
        if not (self._native and k <= 64 and self.world * k <= 512
                and os.environ.get("MPR_SHARDED_NATIVE", "1") != "0"):
            return False
        if not hasattr(self, "_rccl_syms"):
            ok = _lib.ctypes.c_int32(0)
            _lib.call("mpr_rccl_available", _lib.ctypes.byref(ok))
            self._rccl_syms = bool(ok.value)
        return self._rccl_syms and self._comm() != 0

    def _recv_blocks(self, q, B: int, k: int):
        """The native search's receive buffer [n_blocks * B, k, 2] float64 and n_blocks (the
        all_gather fills blocks 0 .. world-1)."""
        return torch.empty((self.world * B, k, 2), device=self.device,
                           dtype=torch.float64), self.world

    def _native_search_all(self, q, k: int):
        """mpr_sharded_search_all on the current stream (q: contiguous fp32 on this device)."""
        B = q.shape[0]
        recv, nb = self._recv_blocks(q, B, k)
        od = torch.empty((B, k), device=self.device, dtype=torch.float32)
        oi = torch.empty((B, k), device=self.device, dtype=torch.int64)
        _lib.call("mpr_sharded_search_all", self._local._h, _lib.c_void_p(self._comm()),
                  self.world, self.rank, _lib.ptr(q), B, int(k), _lib.ptr(recv), nb,
                  _lib.ptr(od), _lib.ptr(oi), _lib.stream_ptr(self.device))
        return od, oi

    def _merge_recv(self, recv, Bp: int, b: int, k: int):
        """Merge the exchanged per-shard top-k, packed [W, Bp, k, 2] float64 (shard w's list
        for query slot j at [w, j]), for query slots 0 .. b-1: (dist, ids) [b, k]."""
        if self._native and k <= 64 and self.world * k <= 512:
            od = torch.empty((b, k), device=self.device, dtype=torch.float32)
            oi = torch.empty((b, k), device=self.device, dtype=torch.int64)
            _lib.call("mpr_topk_merge_packed", _lib.ptr(recv), self.world, Bp, b, k, k,
                      self.metric, _lib.ptr(od), _lib.ptr(oi), _lib.stream_ptr(self.device))
            return od, oi
        d_all, i_all = self._unpack(recv.view(self.world, Bp, k, 2)[:, :b])  # [W, b, k]
        cd = d_all.permute(1, 0, 2).reshape(b, self.world * k)
        ci = i_all.permute(1, 0, 2).reshape(b, self.world * k)
        return self._merge(cd.contiguous(), ci.contiguous(), k)

    def search_all_many(self, queries, k: int):
        """search_all over an iterable of query batches (the same batches on every rank) as a
        pipeline, yielding each batch's (dist, ids) in order, each equal to its search_all: batch
        i+1's local scan is enqueued (on the other of two streams) before batch i's all_gather is
        waited for and merged, so the collective and the merge run behind the next scan instead
        of after it.  Host-staged backends (gloo over device tensors) run them one by one."""
        it = iter(queries)
        if self._host_staged() or self.device.type != "cuda":
            for q in it:
                yield self.search_all(q, k)
            return
        cur = torch.cuda.current_stream(self.device)
        if not hasattr(self, "_streams2"):
            self._streams2 = [torch.cuda.Stream(self.device), torch.cuda.Stream(self.device)]
        streams = self._streams2
        native = self._rccl_ok(k)

        def start(q, j):
            st = streams[j % 2]
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                B = q.shape[0]
                q = q.to(self.device, torch.float32).contiguous()
                # q may be the caller's own tensor (allocated on `cur`): once the caller drops
                # it after the yield, its memory must not be reused while this scan reads it
                q.record_stream(st)
                if native:  # the whole search (RCCL included) enqueued on st in one call
                    return st, B, self._native_search_all(q, k), None
                packed = self._pack(*self._padded_search(q, k))
                recv, work = self._gather(packed, async_op=True)
            return st, B, recv, work

        pend = None
        j = 0
        for q in it:
            nxt = start(q, j)
            j += 1
            if pend is not None:
                yield self._finish_all(pend, k)
            pend = nxt
        if pend is not None:
            yield self._finish_all(pend, k)

    def _finish_all(self, pend, k):
        st, B, recv, work = pend
        if work is None:  # native: recv already holds the merged (dist, ids)
            out = recv
        else:
            with torch.cuda.stream(st):
                work.wait()
                out = self._merge_recv(recv, B, B, k)
        cur = torch.cuda.current_stream(self.device)
        cur.wait_stream(st)
        for t in out:
            t.record_stream(cur)
        return out

    def _padded_search(self, q, k):
        kk = min(k, self.n_local)
        d_loc, i_loc = self._search(q, kk)
        if kk < k:  # tiny shard: pad with sentinels
            pad = k - kk
            fill = float("inf") if self.metric == L2 else float("-inf")
            d_loc = torch.cat([d_loc, torch.full((d_loc.shape[0], pad), fill,
                                                 device=d_loc.device)], 1)
            i_loc = torch.cat([i_loc, torch.full((i_loc.shape[0], pad), -1, dtype=torch.int64,
                                                 device=i_loc.device)], 1)
        return d_loc, i_loc

    def _gather(self, packed, async_op: bool = False):
        """The all_gather of the per-shard top-k, packed [B, k, 2] -> [W B, k, 2] (every rank's
        block, rank-major).  Returns (recv, work or None)."""
        recv = torch.empty((self.world * packed.shape[0],) + tuple(packed.shape[1:]),
                           dtype=packed.dtype, device=packed.device)
        work = dist.all_gather_into_tensor(recv, packed, group=self.group, async_op=async_op)
        return recv, work

    def _pack(self, d, i):
        """(dist, ids) [b, k] -> float64 pairs [b, k, 2] (ids < 2^53, fp32 values exact)."""
        if self._native and d.is_cuda:
            out = torch.empty(tuple(d.shape) + (2,), device=d.device, dtype=torch.float64)
            _lib.call("mpr_topk_pack", _lib.ptr(d.contiguous()), _lib.ptr(i.contiguous()),
                      d.numel(), _lib.ptr(out), _lib.stream_ptr(d.device))
            return out
        return torch.stack([d.to(torch.float64), i.to(torch.float64)], -1).contiguous()

    @staticmethod
    def _unpack(p):
        return p[..., 0].to(torch.float32), p[..., 1].to(torch.int64)
