"""Diagnostic: the C5 projection's pipelined sharded search (bench.ProjectedShard on a world-1
RCCL group) — which exchange path runs, and its ids against the shard's own search."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from multimodalpromptretrieval_amd import synthetic as syn  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
group, _ = bench._world1_group(dev)
n, d, B, k = 1 << 20, 512, 256, 5
g = torch.Generator(device=dev).manual_seed(8)
q = torch.randn((B, d), device=dev, generator=g) * 0.3
for W in (1, 8):
    rows = syn.index_rows_device(7, 0, n // W, d, dev)
    six = bench._projected_shard_class()(rows, dev, W, group)
    print("W", W, "native", six._rccl_ok(k), "comm", hex(six._comm()), flush=True)
    d1, i1 = six._local.search(q, k)
    outs = list(six.search_all_many((q for _ in range(6)), k))
    for j, (dd, ii) in enumerate(outs):
        print(j, bool(torch.equal(ii, i1)), bool(torch.equal(dd, d1)),
              int((ii != i1).sum()), ii[0].tolist(), i1[0].tolist(), flush=True)
    a = six.search_all(q, k)
    print("search_all", bool(torch.equal(a[1], i1)), flush=True)
    del six, rows
    torch.cuda.empty_cache()
