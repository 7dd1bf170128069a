"""predict() latency by MPR_EOS_STOP_CHUNK (0 = one decode graph), alternating runs (dev aid)."""
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
batches = bench.make_batches(4, cfg["B"], dev, seed=100)
res = {}
with torch.no_grad():
    for rep in range(3):
        for chunk in ("0", "2", "4"):
            os.environ["MPR_EOS_STOP_CHUNK"] = chunk
            for i in range(4):
                model.predict(batches[i % 4])
            torch.cuda.synchronize()
            t = time.perf_counter()
            for i in range(30):
                model.predict(batches[i % 4])
            torch.cuda.synchronize()
            res.setdefault(chunk, []).append((time.perf_counter() - t) / 30 * 1e3)
for k, v in res.items():
    print(f"chunk {k}: " + " ".join(f"{x:.2f}" for x in v) + " ms per predict()")
