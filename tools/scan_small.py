"""Small-batch scan timings alone (development aid): the C2 search (6,500 x 1,024, 16 queries,
k = 1) and a 1,048,576 x 512 index searched by 16 queries (k = 5: the two-level merge), timed
with events; MPR_SCAN_SMALL_OFF=1 restores the tile-per-wave scan for the first."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from multimodalpromptretrieval_amd import synthetic as syn  # noqa: E402
from multimodalpromptretrieval_amd.index import DeviceIndex  # noqa: E402

dev = torch.device("cuda:0")
for n, d, b, k in ((6500, 1024, 16, 1), (6500, 1024, 16, 5), (1 << 20, 512, 16, 5)):
    ix = DeviceIndex(syn.index_rows_device(7, 0, n, d, dev), dev)
    q = torch.randn((b, d), device=dev, generator=torch.Generator(device=dev).manual_seed(8)) * 0.3
    for _ in range(3):
        ix.search(q, k)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        ix.search(q, k)
    e1.record()
    torch.cuda.synchronize()
    print(f"n={n} d={d} b={b} k={k}: {1e3 * e0.elapsed_time(e1) / 20:.1f} us per search",
          flush=True)
