"""Greedy decode timing at a given row count (development aid): DeviceT5.generate_padded of
`rows` rows (16-row pieces sharing one decode loop) for t5-small or t5-base, 20 forced steps,
minus the same call with 0 steps = the decode loop alone.  Under
``rocprofv3 --kernel-trace --stats -d <dir> -- python tools/decode_rows.py small 128`` the stats
CSV gives the per-kernel averages of the decode launches.

usage: python tools/decode_rows.py {small|base} ROWS [L] [ITERS]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodalpromptretrieval_amd import synthetic as syn  # noqa: E402
from multimodalpromptretrieval_amd.t5 import DeviceT5  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "small"
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 16
L = int(sys.argv[3]) if len(sys.argv) > 3 else 71
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 20
cfg = syn.T5Config() if which == "small" else syn.T5_BASE
dev = torch.device("cuda:0")
m = DeviceT5(syn.t5_state_dict(3, cfg), dev)
g = torch.Generator().manual_seed(1)
emb = (torch.randn((rows, L, cfg.d_model), generator=g) * 0.3).to(dev)
mask = torch.ones((rows, L), device=dev)


def timed(steps):
    for _ in range(3):
        m.generate_padded(emb, mask, steps)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        m.generate_padded(emb, mask, steps)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


full, enc = timed(20), timed(0)
print(f"t5-{which} {rows} rows L={L}: generate {full:.3f} ms, encoder {enc:.3f} ms, decode "
      f"{full - enc:.3f} ms = {(full - enc) / 20 * 1e3:.1f} us per step", flush=True)
