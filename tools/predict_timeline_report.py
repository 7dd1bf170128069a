"""Summarise a rocprofv3 kernel trace of tools/predict_timeline.py: per predict() call, the
GPU span, busy time, idle gaps and kernel time by kernel family (development aid)."""
import collections
import csv
import glob
import sys

path = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
calls, cur = [], []
for r in rows:
    if cur and int(r["Start_Timestamp"]) - int(cur[-1]["End_Timestamp"]) > 10_000_000:
        calls.append(cur)
        cur = []
    cur.append(r)
calls.append(cur)


def fam(name):
    n = name.replace("void ", "").replace("mpr::(anonymous namespace)::", "")
    return n.split("(")[0].split("<")[0]


for c in calls[-4:]:
    t0, t1 = int(c[0]["Start_Timestamp"]), max(int(r["End_Timestamp"]) for r in c)
    busy = collections.Counter()
    cnt = collections.Counter()
    end = t0
    idle = 0
    for r in c:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s > end:
            idle += s - end
        end = max(end, e)
        busy[fam(r["Kernel_Name"])] += e - s
        cnt[fam(r["Kernel_Name"])] += 1
    print(f"call: span {(t1 - t0) / 1e3:.0f} us, kernels {len(c)}, idle {idle / 1e3:.0f} us")
    for k, v in busy.most_common(12):
        print(f"   {v / 1e3:8.1f} us {cnt[k]:5d}  {k}")
# phases: big gaps inside the last call
c = calls[-1]
prev = None
t0 = int(c[0]["Start_Timestamp"])
for r in c:
    s = int(r["Start_Timestamp"])
    if prev is not None and s - prev > 30_000:
        print(f"  gap {(s - prev) / 1e3:.0f} us at +{(prev - t0) / 1e3:.0f} us before {fam(r['Kernel_Name'])}")
    prev = max(prev or 0, int(r["End_Timestamp"]))
