"""Find where a grouped T5 generate diverges when tower kernels run beside it (DESIGN §9 "Serving-
loop determinism").  Measures nothing; it localises.  Needs MPR_DECODE_TRACE=1 (set here before the
library loads); MPR_DEBUG_GUARD=1 / MPR_DEBUG_LDS_POISON=1 may be added from the environment.

  1. the serving loop's first 8-piece generate call is captured (inputs only);
  2. the call runs alone on slot 1, twice: its decode trace (every decode-chain kernel's output,
     T5Model::trace) must be bit-identical run to run;
  3. it runs N times beside a text-tower pass on the tower stream; each trace is compared with the
     lone one and the FIRST differing segment is reported (kernel, step, layer, how many elements,
     the first one's values), with every earlier segment — that kernel's inputs — identical;
  4. snapshot check: every library buffer is hashed, one tower pass runs alone, the hashes are
     compared (a tower pass may only change the tower workspaces);
  5. MPR_DEBUG_GUARD=1: guard bands checked; MPR_DEBUG_LDS_POISON=1: NaN in the lone trace means a
     chain kernel read LDS it never wrote.

usage: python tools/decode_race.py [runs]"""
import ctypes
import os
import sys

os.environ.setdefault("MPR_DECODE_TRACE", "1")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from multimodalpromptretrieval_amd import _lib, t5  # noqa: E402

KINDS = ["enc_out", "cross_kv", "qkv", "self_att", "o", "cq", "cross_att", "co", "wi", "wo",
         "head_val", "head_idx", "token", "x_next", "ocq", "x1ss", "cowi", "x2ss", "fo",
         "head_rms", "logits"]
INT_KINDS = {"head_idx", "token"}
WS_FIELDS = ["x", "h", "qkv", "ao", "ff", "enc_out", "cross_kv", "cache", "dx", "dq",
             "unfinished", "cur_tok", "enc_in", "mask_in", "part_val", "part_idx", "tok_buf",
             "logits", "mask_enc", "enc_tmp", "ax", "yq", "hz", "x1ss", "x2ss"]


def trace(t5h, slot, dev):
    n, ns = ctypes.c_int64(), ctypes.c_int32()
    _lib.call("mpr_debug_t5_trace", t5h._h, slot, None, 0, ctypes.byref(n), None, 0,
              ctypes.byref(ns), None)
    buf = torch.empty(n.value, dtype=torch.float32, device=dev)
    segs = (ctypes.c_int64 * (6 * ns.value))()
    _lib.call("mpr_debug_t5_trace", t5h._h, slot, _lib.ptr(buf), n.value, ctypes.byref(n), segs,
              ns.value, ctypes.byref(ns), _lib.stream_ptr(dev))
    torch.cuda.synchronize()
    return buf, [tuple(segs[6 * i:6 * i + 6]) for i in range(ns.value)]


def first_diff(ref, cur, segs):
    ne = ref.view(torch.int32) != cur.view(torch.int32)
    if not bool(ne.any()):
        return None
    i0 = int(ne.nonzero()[0, 0])
    for kind, step, layer, rows, cols, off in segs:
        if off <= i0 < off + rows * cols:
            seg_ne = ne[off:off + rows * cols].view(rows, cols)
            r, c = divmod(i0 - off, cols)
            name = KINDS[kind]
            a, b = ref[i0], cur[i0]
            if name in INT_KINDS:
                va, vb = int(a.view(torch.int32)), int(b.view(torch.int32))
            else:
                va, vb = float(a), float(b)
            bad_rows = seg_ne.any(1).nonzero().flatten().tolist()
            return (f"{name} step {step} layer {layer}: {int(seg_ne.sum())} of {rows * cols} "
                    f"elements in rows {bad_rows[:12]}{'...' if len(bad_rows) > 12 else ''}; "
                    f"first [{r}, {c}] {va!r} -> {vb!r}; later segments differing: "
                    f"{int(ne[off + rows * cols:].any())}")
    return f"index {i0} outside every segment"


def explain_cross_att(ref, cur, segs, seg, ins, d_inner, dev):
    """The first differing (row, head) of a cross-attention output: which key's value chunk,
    replaced by what, would explain it (out = sum_k p_k v_k), and where else in cross_kv /
    enc_out that replacement chunk lives."""
    kind, step, layer, rows, cols, off = seg
    D = 64
    out_r = ref[off:off + rows * cols].view(rows, cols)
    out_c = cur[off:off + rows * cols].view(rows, cols)
    ne = (out_r.view(torch.int32) != out_c.view(torch.int32))
    b = int(ne.any(1).nonzero()[0, 0])
    h = int(ne[b].nonzero()[0, 0]) // D
    dims = ne[b, h * D:(h + 1) * D].nonzero().flatten().tolist()
    q_seg = next(s for s in segs if KINDS[s[0]] == "cq" and s[1] == step and s[2] == layer)
    q = ref[q_seg[5]:q_seg[5] + q_seg[3] * q_seg[4]].view(q_seg[3], q_seg[4])[b, h * D:(h + 1) * D]
    kv_seg = next(s for s in segs if KINDS[s[0]] == "cross_kv")
    L = kv_seg[3] // rows
    kv = ref[kv_seg[5]:kv_seg[5] + kv_seg[3] * kv_seg[4]].view(rows, L, kv_seg[4])
    K = kv[b, :, layer * 2 * d_inner + h * D: layer * 2 * d_inner + (h + 1) * D].double()
    V = kv[b, :, layer * 2 * d_inner + d_inner + h * D:
           layer * 2 * d_inner + d_inner + (h + 1) * D].double()
    piece, r = divmod(b, 16)
    m = ins[piece][1][r]
    valid = torch.zeros(L, dtype=torch.bool, device=dev)
    valid[:m.shape[0]] = m != 0
    sc = (K @ q.double()).masked_fill(~valid, float("-inf"))
    p = torch.softmax(sc, 0)
    o64 = p @ V
    dlt = (out_c[b, h * D:(h + 1) * D] - out_r[b, h * D:(h + 1) * D]).double()
    print(f"  row {b} head {h}: differing dims {dims}; ref vs fp64 max err "
          f"{float((out_r[b, h * D:(h + 1) * D].double() - o64).abs().max()):.2e}, delta max "
          f"{float(dlt.abs().max()):.3e}", flush=True)
    # hypothesis: one v_pk_fma_f32 of the P.V sum used the wrong broadcast element of its P pair
    # for the low half (even components): key k's term took P[k ^ 1] instead of P[k], in every
    # lane that ran the instruction (16 lanes of one key group, all 16 dg -> dims 4 dg + e)
    es = sorted(set(dd % 4 for dd in dims))
    if len(es) == 1 and len(dims) == 16:
        e = es[0]
        dd = torch.tensor([4 * g + e for g in range(16)], device=dev)
        best = []
        for k in range(L):
            for kk in (k ^ 1,):
                if kk >= L:
                    continue
                pred = (p[kk] - p[k]) * V[k, dd]
                res = float((pred - dlt[dd]).abs().max())
                best.append((res, k, kk))
        best.sort()
        print(f"  component {e}: best single-term fits (residual, key, key used instead): "
              f"{[(f'{r:.2e}', k, kk) for r, k, kk in best[:3]]}; |delta| {float(dlt[dd].abs().max()):.2e}",
              flush=True)
        return
    ch = sorted(set(dd // 16 for dd in dims))
    for c in ch:
        sl = slice(16 * c, 16 * c + 16)
        best = []
        for k in valid.nonzero().flatten().tolist():
            w = V[k, sl] + dlt[sl] / p[k]
            best.append((float(w.abs().max()), k, w))
        best.sort(key=lambda x: x[0])
        mx, k, w = best[0]
        # where does a chunk equal to w (to 1e-4) live?
        flat = kv.reshape(-1, 16).double()
        dist = (flat - w.view(1, 16)).abs().max(1).values
        j = int(dist.argmin())
        row_j, col_j = divmod(j * 16, kv.shape[2])
        print(f"  dims {16 * c}..{16 * c + 15}: smallest single-key replacement: key {k} "
              f"(p {float(p[k]):.4f}, |w|max {mx:.3f}); nearest cross_kv chunk: row {row_j} "
              f"(b {row_j // L}, key {row_j % L}) col {col_j} (layer {col_j // (2 * d_inner)}, "
              f"{'V' if col_j % (2 * d_inner) >= d_inner else 'K'}, head "
              f"{(col_j % d_inner) // D}, dims {col_j % D}..) at distance {float(dist[j]):.3e}; "
              f"v[{k}] itself at {float((V[k, sl] - w).abs().max()):.3e}", flush=True)


def main():
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    flags = ctypes.c_int32()
    _lib.call("mpr_debug_flags", ctypes.byref(flags))
    print(f"debug flags {flags.value} (1 guard, 2 lds poison, 4 trace)", flush=True)
    cfg = bench.CONFIGS["c2"]
    model, _, _ = bench.build(cfg, dev, None)
    batches = bench.make_batches(16, cfg["B"], seed=100)
    calls = []
    gbp0 = t5.DeviceT5.generate_batches_padded

    def gbp(self, bl, *a, **k):
        if not calls:
            calls.append([(e.clone(), m.clone()) for e, m in bl])
        return gbp0(self, bl, *a, **k)

    t5.DeviceT5.generate_batches_padded = gbp
    with torch.no_grad():
        for _ in model.predict_many(batches, eos_stop=False):
            pass
    t5.DeviceT5.generate_batches_padded = gbp0
    torch.cuda.synchronize()
    ins = calls[0]
    print(f"captured call: {len(ins)} pieces, rows {[e.shape[0] for e, _ in ins]}, "
          f"L {[e.shape[1] for e, _ in ins]}", flush=True)
    t5h = model._device_t5()
    retr = model._retrieval_obj()
    s_img = retr._streams()
    g1 = _lib.role_stream(dev, "gen:1")
    toks = torch.cat([retr.clip_tokenize(b["question"]) for b in batches[:2]])
    if os.environ.get("DR_DEVICE_TOKS") == "1":  # no host-to-device copy inside the tower pass
        toks = toks.to(dev)

    def text_pass(n=3):
        with torch.cuda.stream(s_img):
            for _ in range(n):
                retr.text_encoder.forward(toks)

    def generate():
        with torch.cuda.stream(g1):
            return gbp0(t5h, ins, 20, slot=1)

    with torch.no_grad():
        o_ref = generate()
        torch.cuda.synchronize()  # (the tokens are written on the generate stream)
        o_ref = [x.clone() for x in o_ref]
        ref, segs = trace(t5h, 1, dev)
        print(f"trace: {ref.numel() / 2**20:.1f} M floats in {len(segs)} segments", flush=True)
        n_layers = max(sg[2] for sg in segs) + 1
        d_inner = segs[1][4] // (2 * n_layers)  # the cross_kv segment: Ld * 2 * inner columns
        fl = [i for i, s in enumerate(segs) if KINDS[s[0]] not in INT_KINDS]
        nan_segs = [segs[i] for i in fl
                    if bool(torch.isnan(ref[segs[i][5]:segs[i][5] + segs[i][3] * segs[i][4]]).any())]
        print(f"NaN in the lone trace: {len(nan_segs)} segments "
              f"{[(KINDS[s[0]], s[1], s[2]) for s in nan_segs[:8]]}", flush=True)
        tok_hash = int(torch.cat(o_ref).to(torch.int64).sum()) * 1000003 + \
            int((torch.cat(o_ref).to(torch.int64) * torch.arange(
                torch.cat(o_ref).numel(), device=dev).view_as(torch.cat(o_ref))).sum())
        print(f"lone tokens checksum {tok_hash}", flush=True)
        for r in range(2):
            generate()
            torch.cuda.synchronize()
            cur, _ = trace(t5h, 1, dev)
            print(f"alone rerun {r}: {first_diff(ref, cur, segs) or 'identical'}", flush=True)
        n_diff = 0
        for r in range(runs):
            torch.cuda.synchronize()
            o = generate()
            text_pass()
            torch.cuda.synchronize()
            cur, _ = trace(t5h, 1, dev)
            d = first_diff(ref, cur, segs)
            tok_diff = sum(bool((a != b).any()) for a, b in zip(o_ref, o))
            if d:
                n_diff += 1
                print(f"beside text tower, run {r}: pieces with other tokens {tok_diff}; first "
                      f"difference: {d}", flush=True)
                if d.startswith("cross_att") and n_diff <= 4:
                    ne = ref.view(torch.int32) != cur.view(torch.int32)
                    i0 = int(ne.nonzero()[0, 0])
                    seg = next(sg for sg in segs if sg[5] <= i0 < sg[5] + sg[3] * sg[4])
                    explain_cross_att(ref, cur, segs, seg, ins, d_inner, dev)
        print(f"beside text tower: {n_diff} of {runs} traces differ", flush=True)

        # snapshot: which library buffers does a lone tower pass write?
        def hashes():
            n = ctypes.c_int32()
            _lib.call("mpr_debug_hash_buffers", None, None, None, 0, ctypes.byref(n))
            h = (ctypes.c_uint64 * n.value)()
            p = (ctypes.c_uint64 * n.value)()
            sz = (ctypes.c_int64 * n.value)()
            _lib.call("mpr_debug_hash_buffers", h, p, sz, n.value, ctypes.byref(n))
            return {p[i]: (h[i], sz[i]) for i in range(n.value)}

        names = {}
        for slot in range(6):
            n = ctypes.c_int32()
            p = (ctypes.c_uint64 * 32)()
            sz = (ctypes.c_int64 * 32)()
            _lib.call("mpr_debug_t5_workspace", t5h._h, slot, p, sz, 32, ctypes.byref(n))
            for i in range(n.value):
                if p[i]:
                    names[p[i]] = f"t5 slot {slot} {WS_FIELDS[i]}"
        torch.cuda.synchronize()
        h0 = hashes()
        text_pass(1)
        torch.cuda.synchronize()
        h1 = hashes()
        changed = [(p, h0[p][1]) for p in h0 if p in h1 and h0[p][0] != h1[p][0]]
        print(f"lone text pass changed {len(changed)} of {len(h0)} library buffers; T5 workspace "
              f"ones: {[names[p] for p, _ in changed if p in names]}; sizes "
              f"{sorted(s for _, s in changed)[:20]}", flush=True)
        if flags.value & 1:
            nb = ctypes.c_int32()
            rep = ctypes.create_string_buffer(8192)
            _lib.call("mpr_debug_check_guards", ctypes.byref(nb), rep, 8192)
            print(f"guard bands written: {nb.value}\n{rep.value.decode()}", flush=True)


if __name__ == "__main__":
    main()
