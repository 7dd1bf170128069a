"""The serving loop's stream timeline from hipEvents, without a profiler (development aid: a
rocprofv3 kernel trace serializes the loop's graph launches, so its overlap figures do not hold
for the unprofiled loop).  Timing events around every tower pass (on the tower stream, after its
wait) and every grouped generate call (on its generate stream); prints per-step time, the busy
time of each kind and the time both kinds ran at once.
usage: python tools/loop_events.py [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from multimodalpromptretrieval_amd import dataset, t5  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
cfg = bench.CONFIGS["c2"]
model, _, _ = bench.build(cfg, dev, None)
batches = bench.make_batches(4, cfg["B"], seed=100)
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
marks = []  # (kind, start event, end event)
on = [False]


def wrap(kind, fn):
    def inner(*a, **k):
        if not on[0]:
            return fn(*a, **k)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        out = fn(*a, **k)
        e.record()
        marks.append((kind, s, e))
        return out
    return inner


dataset.encode_towers_multi = wrap("towers", dataset.encode_towers_multi)
t5.DeviceT5.generate_batches_padded = wrap("decode", t5.DeviceT5.generate_batches_padded)
with torch.no_grad():
    for rep in range(3):
        for _ in model.predict_many((batches[i % 4] for i in range(16)), eos_stop=False):
            pass
        torch.cuda.synchronize()
        marks.clear()
        on[0] = True
        base = torch.cuda.Event(enable_timing=True)
        base.record()
        t = time.perf_counter()
        for _ in model.predict_many((batches[i % 4] for i in range(steps)), eos_stop=False):
            pass
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t) * 1e3
        on[0] = False
        iv = {"towers": [], "decode": []}
        for kind, s, e in marks:
            iv[kind].append((base.elapsed_time(s), base.elapsed_time(e)))

        def union(lst):
            out = []
            for a, b in sorted(lst):
                if out and a <= out[-1][1]:
                    out[-1][1] = max(out[-1][1], b)
                else:
                    out.append([a, b])
            return out

        ut, ud = union(iv["towers"]), union(iv["decode"])
        both = sum(max(0.0, min(b1, b2) - max(a1, a2)) for a1, b1 in ut for a2, b2 in ud)
        ua = union(iv["towers"] + iv["decode"])
        span = ua[-1][1] - ua[0][0]
        busy = sum(b - a for a, b in ua)
        bt = sum(b - a for a, b in ut)
        bd = sum(b - a for a, b in ud)
        print(f"{steps} steps: {wall / steps:.3f} ms per step; towers busy {bt:.1f} ms "
              f"({len(iv['towers'])} passes), decode busy {bd:.1f} ms ({len(iv['decode'])} calls),"
              f" both at once {both:.1f} ms; towers or decode running {busy:.1f} of {span:.1f} ms "
              f"({(1 - busy / span) * 100:.1f} % neither), wall {wall:.1f} ms", flush=True)
        if rep == 2:
            for kind in ("towers", "decode"):
                print(kind, " ".join(f"{a:.1f}-{b:.1f}" for a, b in iv[kind][:12]))
