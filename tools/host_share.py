"""Host CPU time vs wall time of the serving loop (development aid): a loop whose host thread is
busy most of the wall time is host-bound, one whose host mostly waits is GPU-bound."""
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
with torch.no_grad():
    for steps in (8, 40, 40):
        torch.cuda.synchronize()
        w, c = time.perf_counter(), time.thread_time()
        for _ in model.predict_many(batches[i % 4] for i in range(steps)):
            pass
        torch.cuda.synchronize()
        w, c = time.perf_counter() - w, time.thread_time() - c
        print(f"{steps} steps: wall {w / steps * 1e3:.3f} ms/step, host thread CPU "
              f"{c / steps * 1e3:.3f} ms/step ({c / w * 100:.0f} %)", flush=True)

if "profile" in sys.argv:
    import cProfile
    import pstats
    pr = cProfile.Profile()
    with torch.no_grad():
        pr.enable()
        for _ in model.predict_many(batches[i % 4] for i in range(40)):
            pass
        torch.cuda.synchronize()
        pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(22)
