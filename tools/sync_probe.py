"""predict() latency alone vs after a serving-loop run (development aid): the bench's
sync_ms_per_step is measured after predict_many; this separates the two."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
cfg = bench.CONFIGS["c2"]
model, _, weights = bench.build(cfg, dev, None)
batches = bench.make_batches(4, cfg["B"], dev, seed=100)


def sync(n=20):
    with torch.no_grad():
        for i in range(3):
            model.predict(batches[i % 4])
        torch.cuda.synchronize()
        t = time.perf_counter()
        for i in range(n):
            model.predict(batches[i % 4])
        torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


print(f"predict() alone: {sync():.2f} ms", flush=True)
if "ib" in sys.argv:
    print("index_build", bench.index_build(cfg, weights, dev)["rows_per_s"], flush=True)
    print(f"predict() after index_build: {sync():.2f} ms", flush=True)
    import gc
    gc.collect()
    torch.cuda.synchronize()
    print(f"predict() after gc: {sync():.2f} ms", flush=True)
with torch.no_grad():
    for _ in model.predict_many(batches[i % 4] for i in range(20)):
        pass
torch.cuda.synchronize()
print(f"predict() after predict_many: {sync():.2f} ms", flush=True)
print(f"predict() again: {sync():.2f} ms", flush=True)
