"""Per-queue kernel counts and cross-queue overlap of a rocprofv3 kernel trace's timed window
(development aid: do the serving loop's streams run concurrently?).
usage: python tools/queue_overlap.py <trace dir>"""
import csv
import glob
import sys

path = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
ts = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r.get("Stream_Id", ""),
       r["Kernel_Name"]) for r in rows]
cuts = [i + 1 for i in range(len(ts) - 1) if ts[i + 1][0] - ts[i][1] > 20_000_000]
segs = [ts[a:b] for a, b in zip([0] + cuts, cuts + [len(ts)])]
win = max(segs, key=len)
by_q = {}
for s, e, q, st, n in win:
    c, t, names = by_q.get(q, (0, 0, {}))
    k = n.split("(")[0].replace("void ", "")[-40:]
    names[k] = names.get(k, 0) + 1
    by_q[q] = (c + 1, t + e - s, names)
for q, (c, t, names) in sorted(by_q.items()):
    top = sorted(names.items(), key=lambda x: -x[1])[:4]
    print(f"queue {q}: {c} kernels, {t / 1e6:.2f} ms; {top}")
streams = {}
for s, e, q, st, n in win:
    streams.setdefault(st, 0)
    streams[st] += 1
print("streams:", streams)
# time with >= 2 kernels running
ev = sorted([(s, 1) for s, e, *_ in win] + [(e, -1) for s, e, *_ in win])
cur, last, multi, busy = 0, ev[0][0], 0, 0
for t, d in ev:
    if cur >= 2:
        multi += t - last
    if cur >= 1:
        busy += t - last
    cur += d
    last = t
print(f"busy {busy / 1e6:.2f} ms, >= 2 kernels at once {multi / 1e6:.2f} ms")
