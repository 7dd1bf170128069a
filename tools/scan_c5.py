"""C5 scan timing alone (development aid): 1,048,576 x 512 index, 256 queries, k = 5; the search
(coarse bf16 + re-rank, or the exact scan with MPR_SCAN_COARSE=0) timed with events."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from multimodalpromptretrieval_amd import synthetic as syn  # noqa: E402
from multimodalpromptretrieval_amd.index import DeviceIndex  # noqa: E402

dev = torch.device("cuda:0")
n, d, k = (1 << 20) // int(sys.argv[1] if len(sys.argv) > 1 else 1), 512, 5
b = int(sys.argv[2]) if len(sys.argv) > 2 else 256
ix = DeviceIndex(syn.index_rows_device(7, 0, n, d, dev), dev)
q = torch.randn((b, d), device=dev, generator=torch.Generator(device=dev).manual_seed(8)) * 0.3
for _ in range(3):
    ix.search(q, k)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    ix.search(q, k)
e1.record()
torch.cuda.synchronize()
_, ids = ix.search(q, k)
tag = "bf2"
print(f"[{tag}] C5 search ({n} rows, {b} queries): {e0.elapsed_time(e1) / 10:.3f} ms, "
      f"exact fallbacks {ix.coarse_fallbacks()}, ids checksum {int(ids.sum())}", flush=True)
