"""Host time of one grouped generate call (mpr_t5_generate_batches, graph replays) against its
GPU time, on an idle GPU (development aid: does the decode graph's launch block the host?).
usage: python tools/launch_block.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
cfg = bench.CONFIGS["c2"]
model, _, _ = bench.build(cfg, dev, None)
batches = bench.make_batches(8, cfg["B"], seed=100)
t5 = model._device_t5()
with torch.no_grad():
    ins = [model.prepare_input(b)[:2] for b in batches]
torch.cuda.synchronize()
from multimodalpromptretrieval_amd import _lib  # noqa: E402

streams = {"default": torch.cuda.current_stream(dev), "torch": torch.cuda.Stream(dev),
           "role gen:0": _lib.role_stream(dev, "gen:0")}
for name, st in streams.items():
    for nb in (8,):
        for steps in (20,):
            with torch.cuda.stream(st):
                for rep in range(3):
                    t5.generate_batches_padded(ins[:nb], steps, slot=0)
                    torch.cuda.synchronize()
                    t = time.perf_counter()
                    t5.generate_batches_padded(ins[:nb], steps, slot=0)
                    th = time.perf_counter() - t
                    torch.cuda.synchronize()
                    tg = time.perf_counter() - t
            print(f"{name}: {nb} batches, {steps} steps: host {th * 1e3:.2f} ms, done "
                  f"{tg * 1e3:.2f} ms", flush=True)
