"""Kernel timeline of single predict() calls (development aid): run under
``rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pt -- python tools/predict_timeline.py``;
predicts are separated by 20 ms host sleeps so the trace splits into calls
(tools/predict_timeline_report.py summarises it)."""
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
batches = bench.make_batches(4, cfg["B"], seed=100)
with torch.no_grad():
    for i in range(12):
        torch.cuda.synchronize()
        time.sleep(0.02)
        t = time.perf_counter()
        model.predict(batches[i % 4])
        torch.cuda.synchronize()
        print(f"predict {i}: {(time.perf_counter() - t) * 1e3:.2f} ms", flush=True)

if "--cprofile" in sys.argv:  # where one predict()'s host time goes
    import cProfile
    import pstats
    with torch.no_grad():
        pr = cProfile.Profile()
        pr.enable()
        for i in range(4):
            model.predict(batches[i % 4])
            torch.cuda.synchronize()
        pr.disable()
    pstats.Stats(pr).sort_stats("cumulative").print_stats(40)
    pstats.Stats(pr).sort_stats("tottime").print_stats(20)
