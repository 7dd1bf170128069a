"""GPU: the serving loop's determinism under concurrency (DESIGN §9 "Determinism").

The reference's greedy decode (architectures/T5VisionModel.py:196-207, called from main.py:262-263)
returns the same tokens for the same inputs.  The serving loop runs a grouped T5 generate on its
generate stream while the next batches' CLIP towers run on the tower stream, so the same call must
return the same tokens whatever shares the chip.  Round 5's bench saw 63/64 answers; the cause was
packed-FP32 VOP3P results corrupted in their low half beside MFMA-heavy waves of another kernel
(tools/decode_race.py localised it to the decode's cross-attention); the library is now built
without packed FP32 ops, and this test is the regression check: 24 calls of the serving loop's
grouped generate (ServingOptions.decode_group pieces: 12 by default; the round-5 loop's 8 when the
test was written), each beside three text-tower passes, all bit-equal to the call run alone (the
old build failed this in 11 of 12 calls with the decode trace on, ~1 in 2 without).
"""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu


def _captured_call(device):
    import bench
    from multimodalpromptretrieval_amd import t5
    cfg = bench.CONFIGS["c2"]
    model, _, _ = bench.build(cfg, device, None)
    batches = bench.make_batches(16, cfg["B"], seed=100)
    calls = []
    gbp0 = t5.DeviceT5.generate_batches_padded

    def gbp(self, bl, *a, **k):
        if not calls:
            calls.append([(e.clone(), m.clone()) for e, m in bl])
        return gbp0(self, bl, *a, **k)

    t5.DeviceT5.generate_batches_padded = gbp
    try:
        with torch.no_grad():
            for _ in model.predict_many(batches, eos_stop=False):
                pass
    finally:
        t5.DeviceT5.generate_batches_padded = gbp0
    torch.cuda.synchronize()
    return model, batches, calls[0]


def test_grouped_generate_bit_identical_beside_tower_passes(device):
    from multimodalpromptretrieval_amd import _lib, serving
    model, batches, ins = _captured_call(device)
    group = serving.ServingOptions.resolve().decode_group
    assert len(ins) == min(group, len(batches)) and all(e.shape[0] == 16 for e, _ in ins)
    t5h = model._device_t5()
    retr = model._retrieval_obj()
    s_img = retr._streams()
    g1 = _lib.role_stream(device, "gen:1")
    toks = torch.cat([retr.clip_tokenize(b["question"]) for b in batches[:2]])

    def generate():
        with torch.cuda.stream(g1):
            return t5h.generate_batches_padded(ins, 20, slot=1)

    with torch.no_grad():
        ref = generate()
        torch.cuda.synchronize()  # (the tokens are written on the generate stream)
        ref = [o.clone() for o in ref]
        differing = []
        for r in range(24):
            out = generate()
            with torch.cuda.stream(s_img):
                for _ in range(3):
                    retr.text_encoder.forward(toks)
            torch.cuda.synchronize()
            n = sum(bool((a != b).any()) for a, b in zip(ref, out))
            if n:
                differing.append((r, n))
    assert not differing, f"(run, pieces with other tokens) beside tower passes: {differing}"
