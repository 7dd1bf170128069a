"""Kernel trace of the serving loop alone (development aid): run under
``rocprofv3 --kernel-trace --output-format csv -d gpurun_out/st -- python tools/serving_trace.py``
then ``python tools/serving_trace.py --report gpurun_out/st``: GPU busy / idle time over the timed
predict_many window (kernels of all streams merged), and the longest idle gaps."""
import glob
import os
import sys
import time

if len(sys.argv) > 2 and sys.argv[1] == "--report":
    import csv
    path = glob.glob(sys.argv[2] + "/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    # the window: between the two long host sleeps the script puts around the timed run
    ts = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    # segments between host sleeps (> 20 ms with no kernel); the timed run has the most kernels
    cuts = [i + 1 for i in range(len(ts) - 1) if ts[i + 1][0] - ts[i][1] > 20_000_000]
    segs = [ts[a:b] for a, b in zip([0] + cuts, cuts + [len(ts)])]
    win = max(segs, key=len)
    t0, t1 = win[0][0], max(e for _, e, _ in win)
    busy, end, last = 0, t0, ""
    idle = []
    for s, e, n in win:
        if s > end:
            idle.append((s - end, (end - t0) / 1e3, n[:60] + "  (after " + last[:50] + ")"))
        busy += max(0, e - max(s, end))
        if e >= end:
            last = n
        end = max(end, e)
    print(f"window {(t1 - t0) / 1e6:.2f} ms, {len(win)} kernels, busy {busy / 1e6:.2f} ms "
          f"({busy / (t1 - t0) * 100:.1f} %), idle {sum(g for g, _, _ in idle) / 1e6:.2f} ms")
    for g, at, n in sorted(idle, reverse=True)[:12]:
        print(f"  idle {g / 1e3:7.1f} us at +{at:8.1f} us before {n}")
    # kernel time by name in the window (sums over overlapping streams: can exceed the window)
    by = {}
    for s, e, n in win:
        k = n.replace("void mpr::(anonymous namespace)::", "").replace("mpr::(anonymous namespace)::", "")
        k = k.split("(mpr::")[0]
        c, t = by.get(k, (0, 0))
        by[k] = (c + 1, t + e - s)
    tot = sum(t for _, t in by.values())
    print(f"kernel time {tot / 1e6:.2f} ms summed over streams")
    for k, (c, t) in sorted(by.items(), key=lambda x: -x[1][1])[:18]:
        print(f"  {t / 1e6:7.2f} ms {t / tot * 100:5.1f} % {c:6d} x {t / c / 1e3:7.2f} us  {k[:70]}")
    sys.exit(0)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
cfg = bench.CONFIGS["c2"]
model, _, _ = bench.build(cfg, dev, None)
batches = bench.make_batches(4, cfg["B"], seed=100)
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
warm = int(sys.argv[2]) if len(sys.argv) > 2 else 8
with torch.no_grad():
    for _ in model.predict_many((batches[i % 4] for i in range(warm)), eos_stop=False):
        pass
    torch.cuda.synchronize()
    time.sleep(0.05)
    t = time.perf_counter()
    for _ in model.predict_many((batches[i % 4] for i in range(steps)), eos_stop=False):
        pass
    torch.cuda.synchronize()
    print(f"{steps} steps: {(time.perf_counter() - t) / steps * 1e3:.3f} ms per step", flush=True)
    time.sleep(0.05)
    torch.zeros(1, device=dev).add_(1)
    torch.cuda.synchronize()
