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
# how the queues interleave: runs of consecutive kernels (start order) from one queue
runs = []
for s, e, q, st, n in win:
    if runs and runs[-1][0] == q:
        runs[-1][1] += 1
        runs[-1][3] = e
    else:
        runs.append([q, 1, s, e])
per_q = {}
for q, c, s, e in runs:
    per_q.setdefault(q, []).append((c, e - s))
for q, lst in sorted(per_q.items()):
    cs = sorted(c for c, _ in lst)
    print(f"queue {q}: {len(lst)} runs, kernels per run median {cs[len(cs) // 2]} max {cs[-1]}, "
          f"longest run {max(d for _, d in lst) / 1e6:.2f} ms")
if len(sys.argv) > 2:  # the run sequence: queue, kernels, start (ms into the window), duration
    t0 = win[0][0]
    for q, c, s, e in runs[:int(sys.argv[2])]:
        print(f"  q{q} {c:5d} kernels at +{(s - t0) / 1e6:7.2f} ms for {(e - s) / 1e6:6.2f} ms")
