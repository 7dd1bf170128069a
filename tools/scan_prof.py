"""Kernel-only scan / merge durations per tools/scan_bench.py shape, from a rocprofv3 kernel
trace of that script (23 searches per shape: 3 warm-up + 20 timed; medians of all 23).

usage: python tools/scan_prof.py <run_kernel_trace.csv>
"""
import csv
import statistics as st
import sys

SHAPES = [(6500, 1024, 16, 1), (10000, 1024, 16, 3), (8192, 1024, 16, 5), (32768, 1024, 16, 5),
          (65536, 1024, 16, 5), (1 << 20, 512, 16, 5), (1 << 20, 512, 256, 5),
          (1 << 17, 512, 256, 5)]


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3  # noqa: E731
    scan = [dur(r) for r in rows if "scan_kernel" in r["Kernel_Name"]
            or "scan_mm_kernel" in r["Kernel_Name"]]
    merge = [dur(r) for r in rows if "merge_kernel" in r["Kernel_Name"]]
    for i, (n, d, b, k) in enumerate(SHAPES):
        s, m = st.median(scan[i * 23:(i + 1) * 23]), st.median(merge[i * 23:(i + 1) * 23])
        gbs = n * d * 4 / (s * 1e-6) / 1e9
        print(f"n={n:8d} d={d:5d} b={b:4d} k={k}: scan {s:8.1f} us ({gbs:6.0f} GB/s index, "
              f"{gbs / 8000:.2f} of 8 TB/s)  merge {m:6.1f} us")


if __name__ == "__main__":
    main()
