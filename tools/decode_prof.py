"""Decode-chain kernel profile: a 16-row t5-small generate (20 steps) replayed N times, for
rocprofv3 --kernel-trace --stats (per-kernel average durations of the decode launches)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodalpromptretrieval_amd import synthetic as syn  # noqa: E402
from multimodalpromptretrieval_amd.t5 import DeviceT5  # noqa: E402

dev = torch.device("cuda:0")
m = DeviceT5(syn.t5_state_dict(3), dev)
g = torch.Generator().manual_seed(1)
emb = (torch.randn((16, 71, 512), generator=g) * 0.3).to(dev)
mask = torch.ones((16, 71), device=dev)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 50
for _ in range(5):
    m.generate_padded(emb, mask, 20)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(n):
    m.generate_padded(emb, mask, 20)
e1.record()
e1.synchronize()
print(f"generate 16 rows x 20 steps: {e0.elapsed_time(e1) / n:.3f} ms", flush=True)
