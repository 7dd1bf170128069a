"""Time the 16-row t5-small greedy decode (bench.py decode_chain's measurement) under the current
environment: one line of JSON with us per decode step (generate of 20 steps minus 0 steps, best of
3 windows of 10 calls), so variants (MPR_ATT_SMALL, MPR_DECODE_FOLD, ...) can be compared in
separate processes: `MPR_ATT_SMALL=wave1 python tools/decode_ab.py`.
usage: python tools/decode_ab.py [rows] [source_len]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from multimodalpromptretrieval_amd import synthetic as syn  # noqa: E402
from multimodalpromptretrieval_amd.t5 import DeviceT5  # noqa: E402


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    L = int(sys.argv[2]) if len(sys.argv) > 2 else 71
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    t5 = DeviceT5(syn.t5_state_dict(3, syn.T5Config()), dev)
    g = torch.Generator().manual_seed(5)
    emb = (torch.randn((rows, L, 512), generator=g) * 0.5).to(dev)
    mask = torch.ones((rows, L), device=dev)

    def timed(n, iters=10):
        t5.generate_padded(emb, mask, n)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(iters):
            t5.generate_padded(emb, mask, n)
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / iters

    full = min(timed(20) for _ in range(3))
    enc = min(timed(0) for _ in range(3))
    toks = t5.generate_padded(emb, mask, 20).cpu()
    env = {k: v for k, v in os.environ.items() if k.startswith("MPR_")}
    print(json.dumps({"env": env, "rows": rows, "L": L, "us_per_step": round((full - enc) * 50, 1),
                      "encoder_ms": round(enc, 3),
                      "tokens_checksum": int((toks.long() * torch.arange(toks.numel()).view_as(
                          toks)).sum())}), flush=True)


if __name__ == "__main__":
    main()
