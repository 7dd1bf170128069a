"""Long host API calls of a rocprofv3 trace (development aid: where does the serving loop's host
block?).  Aligns the HIP API trace with the kernel trace's timed window and lists API calls
longer than a threshold, plus the kernel runs around them.
usage: python tools/api_blocks.py <trace dir> [min_us=300]"""
import csv
import glob
import sys

d = sys.argv[1]
min_ns = int(float(sys.argv[2]) * 1e3) if len(sys.argv) > 2 else 300_000
kp = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
ap = glob.glob(d + "/**/*hip_api_trace.csv", recursive=True)[0]
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"])
             for r in csv.DictReader(open(kp))))
cuts = [i + 1 for i in range(len(ks) - 1) if ks[i + 1][0] - ks[i][1] > 20_000_000]
segs = [ks[a:b] for a, b in zip([0] + cuts, cuts + [len(ks)])]
win = max(segs, key=len)
t0, t1 = win[0][0], max(e for _, e, _ in win)
api = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"])
             for r in csv.DictReader(open(ap)))
api = [a for a in api if t0 - 2_000_000 <= a[0] <= t1]
tot = {}
for s, e, f in api:
    c, t = tot.get(f, (0, 0))
    tot[f] = (c + 1, t + e - s)
print(f"window {(t1 - t0) / 1e6:.2f} ms; API time by function:")
for f, (c, t) in sorted(tot.items(), key=lambda x: -x[1][1])[:12]:
    print(f"  {t / 1e6:8.2f} ms {c:6d} x  {f}")
print(f"calls >= {min_ns / 1e3:.0f} us (start / end relative to the window):")
for s, e, f in api:
    if e - s >= min_ns:
        print(f"  +{(s - t0) / 1e6:8.2f} .. +{(e - t0) / 1e6:8.2f} ms  {f}")
print("graph calls in order (duration ms):")
print("  " + " ".join(f"{'L' if f == 'hipGraphLaunch' else 'I'}{(e - s) / 1e6:.2f}"
                      for s, e, f in api if f in ("hipGraphLaunch", "hipGraphInstantiate")))
