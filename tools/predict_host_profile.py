"""cProfile of single predict() calls (development aid): where the host spends the time the GPU
sits idle between the retrieval copy and the T5 embed.
usage: python tools/predict_host_profile.py [n]"""
import cProfile
import os
import pstats
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
n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
with torch.no_grad():
    for i in range(4):
        model.predict(batches[i % 4])
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i in range(n):
        model.predict(batches[i % 4])
    torch.cuda.synchronize()
    print(f"predict(): {(time.perf_counter() - t) / n * 1e3:.2f} ms", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for i in range(n):
        model.predict(batches[i % 4])
    pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(25)
