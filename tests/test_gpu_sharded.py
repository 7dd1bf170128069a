"""Index sharding on the device kernels: two ranks on one GPU (gloo, the
collectives staged through host memory) hold half the rows each; ``ShardedIndex.search``
(per-rank query blocks of unequal size) and ``ShardedIndex.search_all`` (one query batch on both
ranks) must return exactly the single-index ``DeviceIndex.search`` ids and distances — the
per-shard scans are the same kernels over row subsets and the merge keeps the lowest-global-id
tie rule.  Covers the small-batch scan (b = 16: distances bit-identical too) and the large-batch
coarse path (b = 96: distances within the cdist bound)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

N, D = 5000, 512


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data():
    from multimodalpromptretrieval_amd import synthetic as syn
    X = syn.index_rows(71, N, D)
    X[4000] = X[123]  # an exact duplicate across the shard boundary: ties -> lowest id
    q = syn.index_rows(72, 96, D)
    q[0] = X[123]
    return X, q


def _worker(rank, port, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        from multimodalpromptretrieval_amd.distributed import ShardedIndex
        dev = torch.device("cuda:0")
        X, q = _data()
        six = ShardedIndex(X, dev)
        res = {}
        blocks = [(0, 16), (16, 21)]  # unequal per-rank batches (16 and 5 queries)
        lo, hi = blocks[rank]
        d, i = six.search(q[lo:hi], 5)
        res["search"] = (d.cpu(), i.cpu())
        for b in (16, 96):
            d, i = six.search_all(q[:b], 5)
            res[f"all{b}"] = (d.cpu(), i.cpu())
        out_q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_sharded_search_on_device_equals_single_index(device):
    from multimodalpromptretrieval_amd.index import DeviceIndex
    X, q = _data()
    ix = DeviceIndex(X, device)
    want = {b: tuple(t.cpu() for t in ix.search(q[:b], 5)) for b in (16, 21, 96)}
    del ix
    torch.cuda.synchronize()
    ctx = mp.get_context("spawn")
    out_q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, port, out_q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(out_q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    blocks = [(0, 16), (16, 21)]
    for r in range(2):
        lo, hi = blocks[r]
        d, i = res[r]["search"]
        assert torch.equal(i, want[21][1][lo:hi]) and torch.equal(d, want[21][0][lo:hi])
        d, i = res[r]["all16"]
        assert torch.equal(i, want[16][1]) and torch.equal(d, want[16][0])
        # b = 96 takes the coarse path, whose exact fallback (a shard's own bound decides it)
        # may evaluate a query's keys with the other exact kernel: ids exact, distances within
        # the cdist bound on the squared distance
        d, i = res[r]["all96"]
        assert torch.equal(i, want[96][1]), r
        Xn = (X.double() ** 2).sum(1)[i]
        scale = (q[:96].double() ** 2).sum(1, keepdim=True) + Xn
        assert torch.all((d.double() ** 2 - want[96][0].double() ** 2).abs() <= 2e-6 * scale)
    assert int(want[16][1][0, 0]) == 123 and int(want[16][1][0, 1]) == 4000


def test_search_all_many_pipelined_on_rccl(device):
    """ShardedIndex.search_all_many's two-stream path (batch i+1's scan enqueued before batch
    i's async all_gather is waited for and merged) on a one-rank RCCL group on this GPU: every
    batch equals its search_all (b = 96 and 256 through the coarse path, b = 16 the exact scan),
    with the caller dropping each query tensor as soon as it is handed over (the scan's stream
    keeps it alive).  Then the bench's ProjectedShard (the merge reading W x k candidates) over
    the same pipeline returns the shard's own ids."""
    import sys

    from multimodalpromptretrieval_amd import synthetic as syn
    from multimodalpromptretrieval_amd.distributed import ShardedIndex
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    # keep the in-place ncclAllGather at world 1 (libmpr reads it per call): the RCCL
    # call itself (dlsym'd ncclAllGather on PyTorch's communicator) runs here
    os.environ["MPR_SHARDED_FORCE_COLLECTIVE"] = "1"
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0,
                            world_size=1, device_id=device)
    try:
        X = syn.index_rows(81, 40000, D)
        six = ShardedIndex(X, device)
        assert six._rccl_ok(5), "the native RCCL path (mpr_sharded_search_all) is not available"
        sizes = [96, 16, 256, 96, 16, 256]
        qs = [syn.index_rows(90 + j, b, D) for j, b in enumerate(sizes)]
        want = [tuple(t.cpu() for t in six.search_all(q.to(device), 5)) for q in qs]
        # the native call equals the Python exchange (pack, torch all_gather, packed merge) and
        # the single-index search
        from multimodalpromptretrieval_amd.index import DeviceIndex
        ix = DeviceIndex(X, device)
        os.environ["MPR_SHARDED_NATIVE"] = "0"
        try:
            py = [tuple(t.cpu() for t in six.search_all(q.to(device), 5)) for q in qs]
        finally:
            os.environ.pop("MPR_SHARDED_NATIVE", None)
        for (dw, iw), (dp, ip), q in zip(want, py, qs):
            assert torch.equal(iw, ip) and torch.equal(dw, dp)
            d1, i1 = ix.search(q.to(device), 5)
            assert torch.equal(iw, i1.cpu()) and torch.equal(dw, d1.cpu())

        def fresh():  # each batch a new device tensor, unreferenced by the caller after yield
            for q in qs:
                yield q.to(device)
        got = [tuple(t.cpu() for t in out) for out in six.search_all_many(fresh(), 5)]
        assert len(got) == len(want)
        for j, ((dg, ig), (dw, iw)) in enumerate(zip(got, want)):
            assert torch.equal(ig, iw), j
            assert torch.equal(dg, dw), j
        ps = bench._projected_shard_class()(X.to(device), device, 8)
        q = qs[2].to(device)
        d1, i1 = ps._local.search(q, 5)
        outs = list(ps.search_all_many((q for _ in range(4)), 5))
        for d, i in outs:
            assert torch.equal(i, i1) and torch.equal(d, d1)
    finally:
        os.environ.pop("MPR_SHARDED_FORCE_COLLECTIVE", None)
        dist.destroy_process_group()


def test_native_merge_reads_eight_prefilled_blocks(device):
    """The packed layout a W = 8 exchange hands mpr_sharded_search_all's merge, on one GPU: an
    index of 8 x 2500 rows cut into 8 shards (each a DeviceIndex with its global row offset);
    shards 1-7 are searched and packed into blocks 1-7 of the [8 B, k, 2] receive buffer, and
    shard 0's native call (world 1, rank 0, n_blocks = 8) writes block 0 and merges all eight.
    The result must be the single index's: ids exact (a duplicate row across shards resolves to
    the lower global id), distances bit-identical on the exact scan (b = 16) and within the cdist
    bound on the coarse path (b = 96).  Run with and without the in-place RCCL all_gather (which
    at world 1 must leave blocks 1-7 untouched)."""
    from multimodalpromptretrieval_amd import synthetic as syn
    from multimodalpromptretrieval_amd import _lib
    from multimodalpromptretrieval_amd.distributed import ShardedIndex, shard_bounds
    from multimodalpromptretrieval_amd.index import DeviceIndex
    W, n, k = 8, 8 * 2500, 5
    X = syn.index_rows(83, n, D)
    X[5 * 2500 + 7] = X[11]  # shard 5 holds a copy of a shard-0 row
    X[7 * 2500 + 1] = X[3 * 2500 + 9]
    qs = {b: syn.index_rows(84 + b, b, D) for b in (16, 96)}
    qs[16][0] = X[11]
    qs[96][3] = X[3 * 2500 + 9]
    full = DeviceIndex(X, device)
    want = {b: tuple(t.cpu() for t in full.search(q.to(device), k)) for b, q in qs.items()}
    del full
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0,
                            world_size=1, device_id=device)
    try:
        shards = []
        for r in range(W):
            lo, hi = shard_bounds(n, W, r)
            shards.append(ShardedIndex(X[lo:hi], device, rows_are_local=True, row_offset=lo))
        s0 = shards[0]
        assert s0._rccl_ok(k), "the native RCCL path (mpr_sharded_search_all) is not available"
        for force in ("0", "1"):
            if force == "1":
                os.environ["MPR_SHARDED_FORCE_COLLECTIVE"] = "1"
            for b, q in qs.items():
                qd = q.to(device).contiguous()
                recv = torch.full((W * b, k, 2), float("nan"), device=device, dtype=torch.float64)
                for r in range(1, W):
                    recv[r * b:(r + 1) * b] = shards[r]._pack(*shards[r]._local.search(qd, k))
                foreign = recv[b:].clone()
                od = torch.empty((b, k), device=device, dtype=torch.float32)
                oi = torch.empty((b, k), device=device, dtype=torch.int64)
                _lib.call("mpr_sharded_search_all", s0._local._h, _lib.c_void_p(s0._comm()), 1, 0,
                          _lib.ptr(qd), b, k, _lib.ptr(recv), W, _lib.ptr(od), _lib.ptr(oi),
                          _lib.stream_ptr(device))
                torch.cuda.synchronize()
                assert torch.equal(recv[b:], foreign), (force, b)  # blocks 1-7 untouched
                assert not torch.isnan(recv[:b]).any(), (force, b)  # block 0 written
                dw, iw = want[b]
                assert torch.equal(oi.cpu(), iw), (force, b)
                if b == 16:
                    assert torch.equal(od.cpu(), dw), force
                else:
                    Xn = (X.double() ** 2).sum(1)[iw]
                    scale = (q.double() ** 2).sum(1, keepdim=True) + Xn
                    assert torch.all((od.cpu().double() ** 2 - dw.double() ** 2).abs()
                                     <= 2e-6 * scale), force
            assert int(want[16][1][0, 0]) == 11 and int(want[16][1][0, 1]) == 5 * 2500 + 7
            assert int(want[96][1][3, 0]) == 3 * 2500 + 9
            assert int(want[96][1][3, 1]) == 7 * 2500 + 1
    finally:
        os.environ.pop("MPR_SHARDED_FORCE_COLLECTIVE", None)
        dist.destroy_process_group()
