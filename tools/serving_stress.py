"""The serving loop's answers against predict()'s over many batches, repeated (development aid:
hunting an ordering hazard; run with MPR_EAGER_STREAMS=1 and the MPR_* switches to bisect).
usage: python tools/serving_stress.py [batches] [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
cfg = bench.CONFIGS["c2"]
model, _, _ = bench.build(cfg, dev, None)
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 16
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
batches = bench.make_batches(nb, cfg["B"], seed=100)
with torch.no_grad():
    want = [model.predict(b) for b in batches]
    bad = 0
    for r in range(reps):
        got = list(model.predict_many(batches, eos_stop=False))
        for i, (w, g) in enumerate(zip(want, got)):
            for j, (a, c) in enumerate(zip(w, g)):
                if a != c:
                    bad += 1
                    if bad <= 6:
                        print(f"rep {r} batch {i} row {j}: predict {a[:40]!r} loop {c[:40]!r}")
print(f"{os.environ.get('TAG', '')}: {bad} mismatches over {reps} x {nb} x {cfg['B']} answers",
      flush=True)
