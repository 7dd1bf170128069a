"""Lockstep CLIP-tower timing (development aid): one encode_towers pass (retrieval ViT CLS +
token-feature ViT + CLIP text, bench c2 weights and questions) at several batch sizes, alone on
the device; CUDA events over repeated passes.  Shows how much of a pass is per-launch overhead
and tail (time per image falling with the batch) versus MFMA work.

usage: python tools/towers_bench.py [B ...]   (default 8 16 32 64, then the two-stream test)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402
from multimodalpromptretrieval_amd import encoders  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    model, retr, _ = bench.build(bench.CONFIGS["c2"], dev, None)
    vit_tok = model._device_vit()
    batches = bench.make_batches(4, 16, dev, seed=100)
    sizes = [int(a) for a in sys.argv[1:]] or [8, 16, 32, 64]
    for B in sizes:
        reps = max(1, B // 16)
        img = torch.cat([b["image"] for b in batches] * 4)[:B].contiguous()
        qs = sum([b["question"] for b in batches] * 4, [])[:B]
        toks = retr.clip_tokenize(qs)
        q = torch.empty((B, retr.embed_dim), device=dev)
        di = retr.image_encoder.out_dim

        def run():
            encoders.encode_towers(retr.image_encoder, img, encoders.CLS, out_a=q,
                                   out_a_bstride=retr.embed_dim, vit_b=vit_tok,
                                   mode_b=encoders.TOKENS, text=retr.text_encoder, tokens=toks,
                                   out_t=q[:, di:], out_t_bstride=retr.embed_dim)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        it = 20
        e0.record()
        for _ in range(it):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / it
        print(f"B={B:3d} (x{reps} batches of 16): {ms:7.3f} ms per pass, "
              f"{ms / B * 16:7.3f} ms per 16 images", flush=True)

    if sys.argv[1:]:
        return
    # two batches' passes on two streams at once (second model set: its own workspaces) against
    # the same two passes back to back on one stream
    model2, retr2, _ = bench.build(bench.CONFIGS["c2"], dev, None)
    sets = [(retr, vit_tok), (retr2, model2._device_vit())]
    B = 16
    args = []
    for i, (r, v) in enumerate(sets):
        img = batches[i]["image"].contiguous()
        toks = r.clip_tokenize(batches[i]["question"])
        q = torch.empty((B, r.embed_dim), device=dev)
        args.append((r, v, img, toks, q))

    def one(a):
        r, v, img, toks, q = a
        di = r.image_encoder.out_dim
        encoders.encode_towers(r.image_encoder, img, encoders.CLS, out_a=q,
                               out_a_bstride=r.embed_dim, vit_b=v, mode_b=encoders.TOKENS,
                               text=r.text_encoder, tokens=toks, out_t=q[:, di:],
                               out_t_bstride=r.embed_dim)
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]

    def seq():
        for a in args:
            one(a)

    def conc():
        cur = torch.cuda.current_stream()
        for st, a in zip(streams, args):
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                one(a)
        for st in streams:
            cur.wait_stream(st)
    for name, fn in (("sequential", seq), ("two streams", conc)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        print(f"2 x B=16 passes, {name:11s}: {e0.elapsed_time(e1) / 20:7.3f} ms", flush=True)


if __name__ == "__main__":
    main()
