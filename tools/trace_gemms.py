"""Per-launch GEMM durations from a rocprofv3 kernel trace, grouped by kernel and grid (dev aid).
usage: python tools/trace_gemms.py <run_kernel_trace.csv> [name-substring]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
sub = sys.argv[2] if len(sys.argv) > 2 else "gemm"
agg = collections.defaultdict(list)
for r in rows:
    if sub not in r["Kernel_Name"]:
        continue
    key = (r["Kernel_Name"].split("(")[0][-60:], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"],
           r["Workgroup_Size_X"])
    agg[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = 0
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    v.sort()
    med = v[len(v) // 2]
    tot += sum(v)
    print(f"{k[0]:60s} grid {k[1]:>7}x{k[2]:>4}x{k[3]:>2} wg {k[4]:>4}  n {len(v):5d}  med {med:8.2f} us  sum {sum(v)/1e3:8.2f} ms")
print(f"total {tot/1e3:.2f} ms")
