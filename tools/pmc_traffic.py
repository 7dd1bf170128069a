"""HBM traffic per tiled-GEMM launch of bench.py's roofline replay, from two rocprofv3 --pmc
passes of the same bench command (FETCH_SIZE in one, WRITE_SIZE in the other: they do not fit
one pass on gfx950), windowed to the replay by its two probe_marker_kernel dispatches.

Correction (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7): on gfx950 FETCH_SIZE reports
half of the bytes of a wide coalesced streaming read (the GEMM's operand loads are 16 B per lane),
so read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE x 1024 is taken as is (the epilogue's 4-byte
stores are an uncalibrated width: see the note in the output).

usage: python tools/pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv>
                                   <out.json> [algorithmic_bytes_per_launch]
"""
import csv
import json
import sys


def per_dispatch(path, counter):
    rows = list(csv.DictReader(open(path)))
    disp = {}
    for r in rows:
        if r.get("Counter_Name") != counter:
            continue
        k = int(r["Dispatch_Id"])
        ent = disp.setdefault(k, {"name": r["Kernel_Name"], "v": 0.0})
        ent["v"] += float(r["Counter_Value"])
    order = sorted(disp)
    marks = [k for k in order if "probe_marker_kernel" in disp[k]["name"]]
    if len(marks) < 2:
        raise SystemExit(f"{path}: no replay markers")
    lo, hi = marks[-2], marks[-1]
    vals = [disp[k]["v"] for k in order if lo < k < hi and ("gemm_f32_kernel" in disp[k]["name"] or "gemm_x3_kernel" in disp[k]["name"])]
    return vals


def main():
    fetch = per_dispatch(sys.argv[1], "FETCH_SIZE")
    write = per_dispatch(sys.argv[2], "WRITE_SIZE")
    n = min(len(fetch), len(write))
    fk = sum(fetch) / len(fetch)
    wk = sum(write) / len(write)
    out = {"kernel": "gemm_x3_kernel|gemm_f32_kernel", "window": "bench.py roofline replay (markers)",
           "launches": n, "fetch_size_kb_avg": round(fk, 1), "write_size_kb_avg": round(wk, 1),
           "traffic_bytes_per_launch": round((2.0 * fk + wk) * 1024.0),
           "correction": "read = 2 x FETCH_SIZE (gfx950 half-count of 16 B/lane streaming "
                         "reads); write = WRITE_SIZE (4 B/lane epilogue stores: width "
                         "uncalibrated)",
           "note": "operands of these GEMMs (<= 9.4 MB weights, activations) are largely "
                   "L2/Infinity-Cache resident: FETCH_SIZE counts L2 misses served by the "
                   "Infinity Cache too"}
    if len(sys.argv) > 4:
        alg = float(sys.argv[4])
        out["algorithmic_bytes_per_launch"] = round(alg)
        out["traffic_over_algorithmic"] = round(out["traffic_bytes_per_launch"] / alg, 3)
    print(json.dumps(out))
    with open(sys.argv[3], "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
