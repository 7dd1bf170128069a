"""Idle gaps of a rocprofv3 kernel trace in time order (development aid): every gap of at least
MIN_US microseconds where no kernel of any queue runs, inside the timed window (between the last
two idle stretches of >= 30 ms: the tools' host sleeps around their timed steps), with the
kernels that end before and start after it.  usage: python tools/gap_list.py <trace dir> [MIN_US]"""
import csv
import glob
import sys

d = sys.argv[1]
min_us = float(sys.argv[2]) if len(sys.argv) > 2 else 100.0
rows = []
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
sleeps = []
end = rows[0][1]
for s, e, _ in rows[1:]:
    if s - end >= 30e6:
        sleeps.append((end, s))
    end = max(end, e)
lo, hi = (sleeps[-2][1], sleeps[-1][0]) if len(sleeps) >= 2 else (rows[0][0], end)
end, last = rows[0][1], rows[0][2]
tot = 0.0
for s, e, n in rows[1:]:
    if s > end and lo <= s <= hi and (s - end) / 1e3 >= min_us:
        g = (s - end) / 1e3
        tot += g
        print(f"+{(end - lo) / 1e3:9.1f} us  idle {g:7.1f} us  after {last[:50]:50s} before {n[:50]}")
    if e > end:
        end, last = e, n
print(f"window: {(hi - lo) / 1e3:.1f} us, idle in gaps >= {min_us} us: {tot:.1f} us")
