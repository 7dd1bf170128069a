"""Per-grid GEMM durations inside bench.py's roofline replay window vs outside it (dev aid).
usage: python tools/replay_vs_loop.py <run_kernel_trace.csv> [kernel-substring]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
name = sys.argv[2] if len(sys.argv) > 2 else "gemm_"
marks = [i for i, r in enumerate(rows) if "probe_marker_kernel" in r["Kernel_Name"]]
lo, hi = (marks[-2], marks[-1]) if len(marks) >= 2 else (len(rows), len(rows))
for label, sel in (("replay", rows[lo + 1:hi]), ("outside", rows[:lo] + rows[hi + 1:])):
    agg = collections.defaultdict(list)
    for r in sel:
        if name in r["Kernel_Name"]:
            k = (r["Kernel_Name"].split("<")[1].split(">")[0] if "<" in r["Kernel_Name"] else "",
                 r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
            agg[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"== {label}")
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:12]:
        v.sort()
        print(f"  <{k[0]:28s}> {k[1]:>6}x{k[2]:>3}x{k[3]}  n {len(v):4d} med {v[len(v)//2]:8.2f} "
              f"min {v[0]:8.2f} us")
