"""Summarise a rocprofv3 kernel-trace CSV per (kernel, grid) — development aid.

usage: python tools/prof_summary.py <run_kernel_trace.csv> [steps]
"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = collections.defaultdict(lambda: [0, 0])
    for r in rows:
        n = r["Kernel_Name"].replace("mpr::(anonymous namespace)::", "").split("(")[0]
        n = n.replace("void ", "")[:50]
        key = (n, r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"], r["Workgroup_Size_X"])
        d[key][0] += 1
        d[key][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    tot = sum(v[1] for v in d.values())
    print(f"kernels {len(rows)}  busy {tot / 1e6:.3f} ms  per step {tot / 1e6 / steps:.3f} ms")
    for k, v in sorted(d.items(), key=lambda kv: -kv[1][1])[:40]:
        print(f"{v[1] / tot * 100:5.1f}% {v[1] / 1e6 / steps:7.3f} ms/step "
              f"n={v[0] / steps:6.1f}/step avg={v[1] / v[0] / 1e3:8.2f} us  {k}")


if __name__ == "__main__":
    main()
