"""HBM traffic per tiled-GEMM launch of bench.py's roofline replay, from two rocprofv3 --pmc
passes of the same bench command (FETCH_SIZE in one, WRITE_SIZE in the other: they do not fit
one pass on gfx950), windowed to the replay by its two probe_marker_kernel dispatches.

Correction (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7): on gfx950 FETCH_SIZE reports
half of the bytes of a wide coalesced streaming read (the GEMM's operand loads are 16 B per lane),
so read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE x 1024 is taken as is (the epilogue's 4-byte
stores are an uncalibrated width: see the note in the output).

usage: python tools/pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv>
                                   <out.json> [algorithmic_bytes_per_launch]
       python tools/pmc_traffic.py --sum <dir>   (tools/gemm_pmc.sh's passes p1/ p2/ p3/: every
       counter's mean per dispatch, the effective clock and the wait / issue shares of wave time)
       python tools/pmc_traffic.py --model       (no GPU: the per-XCD L2 traffic model of the
       packed 128x128 kernel's tile order over the serving loop's four grouped tower launches —
       each XCD fetches every A row tile and packed W column tile its run of tiles touches once —
       for the kernel's own band rule and for per-problem band heights; it has no L2 capacity
       term: the bands it picks cut fc2's measured traffic 9 % but raised fc1's / qkv's 2-8 %,
       profiles/r06_x3p_band_ab.txt)
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def per_dispatch(path, counter, by_class=None):
    rows = list(csv.DictReader(open(path)))
    disp = {}
    for r in rows:
        if r.get("Counter_Name") != counter:
            continue
        k = int(r["Dispatch_Id"])
        ent = disp.setdefault(k, {"name": r["Kernel_Name"], "v": 0.0,
                                  "grid": int(r.get("Grid_Size", 0) or 0)})
        ent["v"] += float(r["Counter_Value"])
    order = sorted(disp)
    marks = [k for k in order if "probe_marker_kernel" in disp[k]["name"]]
    if len(marks) < 2:
        raise SystemExit(f"{path}: no replay markers")
    lo, hi = marks[-2], marks[-1]
    sel = [k for k in order if lo < k < hi and any(n in disp[k]["name"] for n in ("gemm_f32_kernel", "gemm_x3_kernel", "gemm_x3p_kernel"))]
    if by_class is not None:  # (kernel template, grid) -> [launches, counter sum]
        for k in sel:
            nm = disp[k]["name"]
            key = (nm[nm.find("gemm_"):nm.find(">") + 1], disp[k]["grid"])
            ent = by_class.setdefault(key, [0, 0.0])
            ent[0] += 1
            ent[1] += disp[k]["v"]
    return [disp[k]["v"] for k in sel]


def sum_passes(root):
    per = defaultdict(lambda: defaultdict(float))  # counter -> dispatch -> value
    dur = {}
    for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            d = int(r["Dispatch_Id"])
            per[r["Counter_Name"]][d] += float(r["Counter_Value"])
            if "End_Timestamp" in r and r.get("Start_Timestamp"):
                dur[(f, d)] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
    mean = {c: sum(v.values()) / max(1, len(v)) for c, v in per.items()}
    for c in sorted(mean):
        print(f"{c:32s} {mean[c]:16.1f}   ({len(per[c])} dispatches)")
    if dur:
        print(f"{'duration_us (profiled)':32s} {sum(dur.values()) / len(dur):16.2f}")
    g = mean.get("GRBM_GUI_ACTIVE")
    if g and dur:
        us = sum(dur.values()) / len(dur)
        print(f"effective clock GHz (GRBM_GUI_ACTIVE / 8 XCD / duration): {g / 8 / us * 1e-3:.3f}")
    w, b = mean.get("SQ_WAVE_CYCLES"), mean.get("SQ_BUSY_CYCLES")
    m = mean.get("SQ_VALU_MFMA_BUSY_CYCLES")
    if m and b:
        print(f"MFMA busy / (SQ_BUSY_CYCLES x 4 SIMD x 32 CU per SE...): raw ratio {m / b:.3f}")
    if w:
        for c in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM", "SQ_WAIT_INST_LDS"):
            if c in mean:
                print(f"{c} / SQ_WAVE_CYCLES = {mean[c] / w:.3f}")



def _cdiv(a, b):
    return -(-a // b)


def _tile(t, gy, gx, G):  # gemm_x3p_kernel's band order: (bx, by) of a problem's tile t
    full, band = gy // G * G, G * gx
    if t < (full // G) * band:
        gb, tt = divmod(t, band)
        bx = tt // G
        return bx, gb * G + tt - bx * G
    rem, tt = gy - full, t - (full // G) * band
    return tt // rem, full + tt - (tt // rem) * rem


def model_traffic(probs, bands=None, B=128):
    """Bytes one launch's XCDs fetch beyond L2 (A row tiles fp32, packed W column tiles 6 B per
    element, each once per XCD that touches it) + C written once; bands=None: the kernel's rule."""
    total = sum(_cdiv(M, B) * _cdiv(N, B) for M, N, K in probs)
    q, r = divmod(total, 8)
    run = (total + 7) >> 3
    g0 = int(run ** 0.5)
    while (g0 + 1) ** 2 <= run:
        g0 += 1
    xcd = lambda t: t // (q + 1) if t < r * (q + 1) else r + (t - r * (q + 1)) // max(q, 1)
    seen, off, byts = set(), 0, 0
    for z, (M, N, K) in enumerate(probs):
        gy, gx = _cdiv(M, B), _cdiv(N, B)
        G = min(bands[z] if bands else g0, gy)
        for t in range(gy * gx):
            bx, by = _tile(t, gy, gx, G)
            x = xcd(off + t)
            for key, b in ((("A", x, z, by), min(B, M - by * B) * K * 4),
                           (("W", x, z, bx), min(B, N - bx * B) * K * 6)):
                if key not in seen:
                    seen.add(key)
                    byts += b
        off += gy * gx
    return byts + sum(M * N * 4 for M, N, K in probs)


def model_main():
    launches = {"qkv": [(1600, 2304, 768)] * 2 + [(400, 1536, 512), (384, 1536, 512)],
                "out": [(1600, 768, 768)] * 2 + [(400, 512, 512), (384, 512, 512)],
                "fc1": [(1600, 3072, 768)] * 2 + [(400, 2048, 512), (384, 2048, 512)],
                "fc2": [(1600, 768, 3072)] * 2 + [(400, 512, 2048), (384, 512, 2048)]}
    tot = [0, 0, 0]
    for name, probs in launches.items():
        alg = sum(M * K * 4 + N * K * 4 + M * N * 4 for M, N, K in probs)
        bands = []
        for z in range(len(probs)):  # each problem's band height alone (the others' costs fixed)
            gy = _cdiv(probs[z][0], 128)
            bands.append(min(range(1, gy + 1), key=lambda G: model_traffic(
                probs, [*bands, G, *[1] * (len(probs) - z - 1)])))
        own, tuned = model_traffic(probs), model_traffic(probs, bands)
        tot[0] += alg; tot[1] += own; tot[2] += tuned
        print(f"{name}: algorithmic {alg / 1e6:.1f} MB, kernel rule {own / 1e6:.1f} "
              f"({own / alg:.2f}x), bands {bands} {tuned / 1e6:.1f} ({tuned / alg:.2f}x)")
    print(f"all four: kernel rule {tot[1] / tot[0]:.2f}x, per-problem bands {tot[2] / tot[0]:.2f}x")


def main():
    if sys.argv[1] == "--sum":
        return sum_passes(sys.argv[2])
    if sys.argv[1] == "--model":
        return model_main()
    fc, wc = {}, {}
    fetch = per_dispatch(sys.argv[1], "FETCH_SIZE", fc)
    write = per_dispatch(sys.argv[2], "WRITE_SIZE", wc)
    n = min(len(fetch), len(write))
    fk = sum(fetch) / len(fetch)
    wk = sum(write) / len(write)
    out = {"kernel": "gemm_x3p_kernel|gemm_x3_kernel|gemm_f32_kernel", "window": "bench.py roofline replay (markers)",
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
    # per (kernel, grid) class: launches, MB per launch (2 x FETCH + WRITE), share of the total
    tot = sum(2 * v[1] + wc.get(k, [0, 0.0])[1] for k, v in fc.items())
    out["classes"] = [{"kernel": k[0], "grid": k[1], "launches": v[0],
                       "mb_per_launch": round((2 * v[1] + wc.get(k, [0, 0.0])[1]) * 1024 / v[0] / 1e6, 2),
                       "share": round((2 * v[1] + wc.get(k, [0, 0.0])[1]) / tot, 3)}
                      for k, v in sorted(fc.items(), key=lambda x: -(2 * x[1][1]))][:16]
    print(json.dumps({k: v for k, v in out.items() if k != "classes"}))
    with open(sys.argv[3], "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
