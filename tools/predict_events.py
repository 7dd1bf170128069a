"""One predict() at a time, stage by stage, from hipEvents and host clocks (development aid; no
profiler: rocprofv3's kernel trace blocks the host inside graph launches).  Stages: the paired
towers, the index search, the T5 generate; prints each stage's GPU time and the GPU-idle gaps
between them (host work: top-k sync, prompts, tokenizer, launches).
usage: python tools/predict_events.py [calls]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from multimodalpromptretrieval_amd import dataset, index, t5  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
cfg = bench.CONFIGS["c2"]
model, _, _ = bench.build(cfg, dev, None)
batches = bench.make_batches(4, cfg["B"], seed=100)
calls = int(sys.argv[1]) if len(sys.argv) > 1 else 12
marks = []


def wrap(kind, fn):
    def inner(*a, **k):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        h0 = time.perf_counter()
        out = fn(*a, **k)
        h1 = time.perf_counter()
        e.record()
        marks.append((kind, s, e, h0, h1))
        return out
    return inner


dataset.encode_towers = wrap("towers", dataset.encode_towers)
index.DeviceIndex.search = wrap("search", index.DeviceIndex.search)
t5.DeviceT5.generate = wrap("generate", t5.DeviceT5.generate)
rows = []
with torch.no_grad():
    for i in range(calls):
        torch.cuda.synchronize()
        time.sleep(0.01)
        marks.clear()
        base = torch.cuda.Event(enable_timing=True)
        base.record()
        t = time.perf_counter()
        model.predict(batches[i % 4])
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t) * 1e3
        st = {k: (base.elapsed_time(s), base.elapsed_time(e), (h1 - h0) * 1e3)
              for k, s, e, h0, h1 in marks}
        rows.append((wall, st))
for wall, st in rows[2:]:
    tw, se, ge = st["towers"], st["search"], st["generate"]
    print(f"wall {wall:6.2f} ms | towers {tw[0]:5.2f}-{tw[1]:5.2f} | search {se[0]:5.2f}-{se[1]:5.2f}"
          f" | gap {ge[0] - se[1]:5.2f} | generate {ge[0]:5.2f}-{ge[1]:5.2f} ({ge[1] - ge[0]:5.2f},"
          f" host {ge[2]:5.2f}) | tail {wall - ge[1]:5.2f}", flush=True)
