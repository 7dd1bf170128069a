"""Where does the serving loop's run-to-run variation enter (development aid)?  Runs predict_many
over the same batches several times, keeping device copies of every grouped generate call's
inputs (embeds, masks) and outputs (tokens), then compares the reps call by call.
usage: python tools/serving_stress2.py [batches] [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from multimodalpromptretrieval_amd import t5  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
cfg = bench.CONFIGS["c2"]
model, _, _ = bench.build(cfg, dev, None)
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 24
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
batches = bench.make_batches(nb, cfg["B"], seed=100)
calls = []
_gbp = t5.DeviceT5.generate_batches_padded


def gbp(self, bl, *a, **k):
    ins = [(e.clone(), m.clone()) for e, m in bl]
    outs = _gbp(self, bl, *a, **k)
    calls.append((ins, [o.clone() for o in outs]))
    return outs


t5.DeviceT5.generate_batches_padded = gbp
runs = []
with torch.no_grad():
    for _ in model.predict_many(batches[:8], eos_stop=False):
        pass
    for r in range(reps):
        calls.clear()
        ans = list(model.predict_many(batches, eos_stop=False))
        torch.cuda.synchronize()
        runs.append((ans, list(calls)))
a0, c0 = runs[0]
for r in range(1, reps):
    a, c = runs[r]
    diff_ans = [(i, j) for i in range(nb) for j in range(cfg["B"]) if a[i][j] != a0[i][j]]
    msg = []
    for ci, ((ins0, outs0), (ins1, outs1)) in enumerate(zip(c0, c)):
        de = [bool((e0 != e1).any()) for (e0, _), (e1, _) in zip(ins0, ins1)]
        dm = [bool((m0 != m1).any()) for (_, m0), (_, m1) in zip(ins0, ins1)]
        do = [bool((o0 != o1).any()) for o0, o1 in zip(outs0, outs1)]
        if any(de) or any(dm) or any(do):
            msg.append(f"call {ci}: embeds differ {[i for i, x in enumerate(de) if x]}, masks "
                       f"{[i for i, x in enumerate(dm) if x]}, tokens {[i for i, x in enumerate(do) if x]}")
    print(f"rep {r} vs rep 0: {len(diff_ans)} answers differ {diff_ans[:6]}; " + ("; ".join(msg) or "calls identical"), flush=True)

# the same call's inputs replayed: alone on one stream (synchronised), then two calls at once on
# slots 0 and 1 on the two generate streams
from multimodalpromptretrieval_amd import _lib  # noqa: E402

t5h = model._device_t5()
ins1, outs1 = c0[1]
ins0, _ = c0[0]
ref = None
alone = []
with torch.no_grad():
    for r in range(6):
        o = t5.DeviceT5.generate_batches_padded.__wrapped__(t5h, ins1, 20, slot=1) \
            if hasattr(t5.DeviceT5.generate_batches_padded, "__wrapped__") else _gbp(t5h, ins1, 20, slot=1)
        torch.cuda.synchronize()
        alone.append([x.clone() for x in o])
    print("alone:", [[bool((a != b).any()) for a, b in zip(alone[0], x)] for x in alone[1:]])
    g0, g1 = _lib.role_stream(dev, "gen:0"), _lib.role_stream(dev, "gen:1")
    conc = []
    for r in range(6):
        torch.cuda.synchronize()
        with torch.cuda.stream(g0):
            _gbp(t5h, ins0, 20, slot=0)
        with torch.cuda.stream(g1):
            o = _gbp(t5h, ins1, 20, slot=1)
        torch.cuda.synchronize()
        conc.append([x.clone() for x in o])
    print("concurrent vs alone:", [[bool((a != b).any()) for a, b in zip(alone[0], x)] for x in conc])
    # the call beside a tower pass + scan (retrieval prefetch of two other batches) on the tower
    # stream, repeated
    tw = []
    for r in range(8):
        torch.cuda.synchronize()
        with torch.cuda.stream(g1):
            o = _gbp(t5h, ins1, 20, slot=1)
        pres = model._prefetch(batches[2 * (r % 4):2 * (r % 4) + 2], 0)
        torch.cuda.synchronize()
        tw.append([x.clone() for x in o])
        for b in batches[2 * (r % 4):2 * (r % 4) + 2]:  # drop the prefetched entries
            model._retrieval_obj()._prefetched.pop(model._retrieval_obj()._key(b), None)
    print("beside towers vs alone:", [[bool((a != b).any()) for a, b in zip(alone[0], x)] for x in tw])
    retr = model._retrieval_obj()
    vit = model._device_vit()
    from multimodalpromptretrieval_amd.encoders import encode_towers_multi, CLS, TOKENS  # noqa
    s_img = retr._streams()
    imgs = torch.cat([batches[0]["image"], batches[1]["image"]]).to(dev)
    toks = [retr.clip_tokenize(b["question"]) for b in batches[:2]]
    qx = torch.randn(32, 1024, device=dev)

    def towers():
        with torch.cuda.stream(s_img):
            encode_towers_multi(retr.image_encoder, imgs, CLS, vit_b=vit, mode_b=TOKENS,
                                text=retr.text_encoder, tokens=toks, slot=0)

    def scan():
        with torch.cuda.stream(s_img):
            for _ in range(20):
                retr.index.search(qx, 1)

    for name, fn in (("towers only", towers), ("scan only", scan)):
        res = []
        for r in range(int(os.environ.get("STRESS_N", "12"))):
            torch.cuda.synchronize()
            with torch.cuda.stream(g1):
                o = _gbp(t5h, ins1, 20, slot=1)
            fn()
            torch.cuda.synchronize()
            res.append(sum(bool((a != b).any()) for a, b in zip(alone[0], o)))
        print(f"beside {name}: pieces differing per run {res}", flush=True)
    # the T5 encoder alone (mpr_t5_encode) beside tower passes: 16 rows, or every piece of the
    # call stacked (STRESS_ENC_ALL=1: the 128-row launches take the 128x128 tiles)
    e1, m1 = ins1[0]
    if os.environ.get("STRESS_ENC_ALL") == "1":
        Lm = max(e.shape[1] for e, _ in ins1)
        e1 = torch.cat([torch.nn.functional.pad(e, (0, 0, 0, Lm - e.shape[1])) for e, _ in ins1])
        m1 = torch.cat([torch.nn.functional.pad(m, (0, Lm - m.shape[1])) for _, m in ins1])
    with torch.cuda.stream(g1):
        enc_ref = t5h.encode(e1, m1).clone()
    torch.cuda.synchronize()
    res = []
    for r in range(16):
        with torch.cuda.stream(g1):
            outs_e = [t5h.encode(e1, m1) for _ in range(4)]
        towers()
        towers()
        torch.cuda.synchronize()
        res.append(sum(bool((x != enc_ref).any()) for x in outs_e))
    print(f"T5 encoder beside towers: outputs differing per run (of 4) {res}", flush=True)
    # one tower pass beside the decode, the tower outputs compared run to run
    def towers_out():
        with torch.cuda.stream(s_img):
            a, b, t = encode_towers_multi(retr.image_encoder, imgs, CLS, vit_b=vit, mode_b=TOKENS,
                                          text=retr.text_encoder, tokens=toks, slot=0)
        return a, b, t
    ta, tb, tt = [x.clone() if torch.is_tensor(x) else [y.clone() for y in x] for x in towers_out()]
    torch.cuda.synchronize()
    res = []
    for r in range(12):
        with torch.cuda.stream(g1):
            _gbp(t5h, ins1, 20, slot=1)
        a, b, t = towers_out()
        torch.cuda.synchronize()
        res.append((bool((a != ta).any()), bool((b != tb).any()),
                    any(bool((x != y).any()) for x, y in zip(t, tt))))
    print(f"towers beside a decode: (CLS, tokens, text) differ per run {res}", flush=True)
    # encoder + cross K/V + teacher-forced decoder (mpr_t5_logits) over every piece stacked,
    # beside tower passes
    Lm = max(e.shape[1] for e, _ in ins1)
    eall = torch.cat([torch.nn.functional.pad(e, (0, 0, 0, Lm - e.shape[1])) for e, _ in ins1])
    mall = torch.cat([torch.nn.functional.pad(m, (0, Lm - m.shape[1])) for _, m in ins1])
    dec_ids = torch.zeros((eall.shape[0], 8), dtype=torch.long)
    with torch.cuda.stream(g1):
        lref = t5h.logits(eall, mall, dec_ids).clone()
    torch.cuda.synchronize()
    res = []
    for r in range(16):
        with torch.cuda.stream(g1):
            lo = [t5h.logits(eall, mall, dec_ids) for _ in range(2)]
        towers()
        towers()
        torch.cuda.synchronize()
        res.append(sum(bool((x != lref).any()) for x in lo))
    print(f"T5 logits (tf) beside towers: outputs differing per run (of 2) {res}", flush=True)
    # the grouped generate over the first k pieces only, beside tower passes
    for k in (1, 2, 8):
        sub = ins1[:k]
        with torch.cuda.stream(g1):
            ref = [x.clone() for x in _gbp(t5h, sub, 20, slot=1)]
        torch.cuda.synchronize()
        res = []
        for r in range(int(os.environ.get("STRESS_N", "12"))):
            with torch.cuda.stream(g1):
                o = _gbp(t5h, sub, 20, slot=1)
            towers()
            torch.cuda.synchronize()
            res.append(sum(bool((a != b).any()) for a, b in zip(ref, o)))
        print(f"generate over {k} pieces beside towers: pieces differing {res}", flush=True)
    # one piece's generate beside other workloads on the tower stream
    def enc_big():
        with torch.cuda.stream(s_img):
            for _ in range(3):
                t5h.encode(eall, mall)

    big = torch.randn(4096, 4096, device=dev)

    def mm_big():
        with torch.cuda.stream(s_img):
            for _ in range(6):
                torch.mm(big, big)

    sub = ins1[:1]
    with torch.cuda.stream(g1):
        ref = [x.clone() for x in _gbp(t5h, sub, 20, slot=1)]
    torch.cuda.synchronize()
    for name, fn in (("T5 encoder x3", enc_big), ("torch mm 4096^3 x6", mm_big), ("towers", towers)):
        res = []
        for r in range(int(os.environ.get("STRESS_N", "12"))):
            with torch.cuda.stream(g1):
                o = _gbp(t5h, sub, 20, slot=1)
            fn()
            torch.cuda.synchronize()
            res.append(sum(bool((a != b).any()) for a, b in zip(ref, o)))
        print(f"1-piece generate beside {name}: differing {sum(res)} of {len(res)}", flush=True)
    # the 8-piece generate beside one tower at a time
    tok_all = torch.cat(toks)

    def vit_only():
        with torch.cuda.stream(s_img):
            vit.forward(imgs, TOKENS)
            retr.image_encoder.forward(imgs, CLS)

    def text_only():
        with torch.cuda.stream(s_img):
            for _ in range(3):
                retr.text_encoder.forward(tok_all)

    with torch.cuda.stream(g1):
        ref = [x.clone() for x in _gbp(t5h, ins1, 20, slot=1)]
    torch.cuda.synchronize()
    for name, fn in (("ViTs", vit_only), ("text tower", text_only), ("towers", towers)):
        res = []
        for r in range(int(os.environ.get("STRESS_N", "12"))):
            with torch.cuda.stream(g1):
                o = _gbp(t5h, ins1, 20, slot=1)
            fn()
            torch.cuda.synchronize()
            res.append(sum(bool((a != b).any()) for a, b in zip(ref, o)))
        print(f"8-piece generate beside {name}: differing {sum(res)} pieces over {len(res)} runs",
              flush=True)
    # the grouped generate's pieces through the T5 encoder alone, and the teacher-forced logits,
    # beside the text tower
    with torch.cuda.stream(g1):
        eref = t5h.encode(eall, mall).clone()
        lref2 = t5h.logits(eall, mall, dec_ids).clone()
    torch.cuda.synchronize()
    re, rl = [], []
    for r in range(int(os.environ.get("STRESS_N", "12"))):
        with torch.cuda.stream(g1):
            e_ = t5h.encode(eall, mall)
            l_ = t5h.logits(eall, mall, dec_ids)
        text_only()
        torch.cuda.synchronize()
        re.append(bool((e_ != eref).any()))
        rl.append(bool((l_ != lref2).any()))
    print(f"beside the text tower: encoder outputs differing {sum(re)} / {len(re)}, logits {sum(rl)} / {len(rl)}", flush=True)
    # the 8-piece generate beside the T5 encoder's own split-bf16 launches (3 passes of 128 rows)
    res = []
    for r in range(int(os.environ.get("STRESS_N", "12"))):
        with torch.cuda.stream(g1):
            o = _gbp(t5h, ins1, 20, slot=1)
        enc_big()
        torch.cuda.synchronize()
        res.append(sum(bool((a != b).any()) for a, b in zip(ref, o)))
    print(f"8-piece generate beside the T5 encoder: differing {sum(res)} pieces over {len(res)} runs", flush=True)
    # the 8-piece generate beside raw packed-W GEMM launches of given shapes (mpr_gemm_f32_packed)
    def packed_gemm_fn(M, N, K, act=0):
        A = torch.randn(M, K, device=dev)
        W = torch.randn(N, K, device=dev) * 0.05
        nbytes = _lib.c_int64()
        _lib.call("mpr_pack_x3_bytes", N, K, _lib.ctypes.byref(nbytes))
        img = torch.empty(nbytes.value, dtype=torch.uint8, device=dev)
        _lib.call("mpr_pack_x3", _lib.ptr(W), N, K, K, _lib.ptr(img), nbytes.value, _lib.stream_ptr())
        C = torch.empty(M, N, device=dev)

        def fn():
            with torch.cuda.stream(s_img):
                for _ in range(12):
                    _lib.call("mpr_gemm_f32_packed", _lib.ptr(A), K, _lib.ptr(W), K, _lib.ptr(img),
                              _lib.ptr(C), N, M, N, K, None, 0, act, _lib.stream_ptr(dev))
        return fn

    shapes = ((2464, 512, 2048, 0), (2464, 1536, 512, 0), (800, 2304, 768, 0))
    for shape in shapes:
        fn = packed_gemm_fn(*shape)
        res = []
        for r in range(int(os.environ.get("STRESS_N", "12"))):
            with torch.cuda.stream(g1):
                o = _gbp(t5h, ins1, 20, slot=1)
            fn()
            torch.cuda.synchronize()
            res.append(sum(bool((a != b).any()) for a, b in zip(ref, o)))
        print(f"8-piece generate beside packed GEMM {shape}: differing {sum(res)} pieces over {len(res)} runs", flush=True)
