"""The C5 projection's W = 8 per-rank pipelined search (bench.ProjectedShard: the product's
ShardedIndex.search_all_many on a world-1 RCCL group, merging 8 x 5 candidates per query):
GPU time per batch (hipEvents), the host's enqueue time per batch, and the one-GPU DeviceIndex
search on two alternating streams for comparison.  Run under rocprofv3 --kernel-trace --stats
for the per-kernel split.  usage: python tools/proj_trace.py [W] [batches]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from multimodalpromptretrieval_amd import synthetic as syn  # noqa: E402
from multimodalpromptretrieval_amd.index import DeviceIndex  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else 8
NB = int(sys.argv[2]) if len(sys.argv) > 2 else 40
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
group, _ = bench._world1_group(dev)
n, d, B, k = 1 << 20, 512, 256, 5
g = torch.Generator(device=dev).manual_seed(8)
q = torch.randn((B, d), device=dev, generator=g) * 0.3
rows = syn.index_rows_device(7, 0, n // W, d, dev)
six = bench._projected_shard_class()(rows, dev, W, group)
print("native", six._rccl_ok(k), flush=True)
for rep in range(3):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    t0 = time.perf_counter()
    for _ in six.search_all_many((q for _ in range(NB)), k):
        pass
    th = time.perf_counter() - t0
    e1.record()
    e1.synchronize()
    print(f"search_all_many W={W}: {e0.elapsed_time(e1) / NB * 1e3:.1f} us per batch GPU, "
          f"host enqueue {th / NB * 1e6:.1f} us per batch", flush=True)
ix = six._local
streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
cur = torch.cuda.current_stream(dev)
for rep in range(3):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for st in streams:
        st.wait_stream(cur)
    t0 = time.perf_counter()
    for i in range(NB):
        with torch.cuda.stream(streams[i % 2]):
            ix.search(q, k)
    th = time.perf_counter() - t0
    for st in streams:
        cur.wait_stream(st)
    e1.record()
    e1.synchronize()
    print(f"DeviceIndex.search two streams: {e0.elapsed_time(e1) / NB * 1e3:.1f} us per batch, "
          f"host {th / NB * 1e6:.1f} us", flush=True)
