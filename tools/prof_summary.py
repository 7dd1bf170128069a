"""Summarise a rocprofv3 kernel-trace CSV per (kernel, grid) — development aid — and, with
--replay, the tiled-GEMM launches inside bench.py's roofline replay (between the two
probe_marker_kernel dispatches), the number bench.py's ``roofline.avg_launch_us`` must agree
with.

usage: python tools/prof_summary.py <run_kernel_trace.csv> [steps]
       python tools/prof_summary.py --replay <run_kernel_trace.csv> [out.json]
"""
import collections
import csv
import json
import sys


def _rows(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return rows


def replay_window(rows, names=("gemm_x3_kernel", "gemm_x3p_kernel", "gemm_f32_kernel"), marker="probe_marker_kernel"):
    marks = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    if len(marks) < 2:
        raise SystemExit("no replay markers in the trace (bench.py run without --no-probe?)")
    lo, hi = marks[-2], marks[-1]
    return [r for r in rows[lo + 1:hi] if any(n in r["Kernel_Name"] for n in names)]


def main():
    if sys.argv[1] == "--replay":
        rows = replay_window(_rows(sys.argv[2]))
        durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]
        out = {"kernel": "gemm_x3p_kernel|gemm_x3_kernel|gemm_f32_kernel", "window": "bench.py roofline replay (markers)",
               "launches": len(durs), "avg_launch_us": round(sum(durs) / len(durs) / 1e3, 3),
               "total_ms": round(sum(durs) / 1e6, 4)}
        print(json.dumps(out))
        if len(sys.argv) > 3:
            with open(sys.argv[3], "w") as f:
                json.dump(out, f, indent=1)
        return
    path = sys.argv[1]
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    rows = _rows(path)
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
