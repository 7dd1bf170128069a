"""Standalone T5 generate timing split (development aid): encoder-only (max_new 0) vs 20-step
generate at B rows, t5-small or t5-base, hipEvents on the caller's stream; run under
`rocprofv3 --kernel-trace --stats` for per-kernel durations with nothing else on the chip.
usage: python tools/decode_split.py [B] [L] [small|base]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from multimodalpromptretrieval_amd import synthetic as syn  # noqa: E402
from multimodalpromptretrieval_amd.t5 import DeviceT5  # noqa: E402


def timed(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    L = int(sys.argv[2]) if len(sys.argv) > 2 else 71
    size = sys.argv[3] if len(sys.argv) > 3 else "small"
    dev = torch.device("cuda:0")
    cfg = syn.T5Config() if size == "small" else syn.T5_BASE
    t5 = DeviceT5(syn.t5_state_dict(2, cfg), dev)
    emb = torch.randn(B, L, cfg.d_model, device=dev) * 0.05
    mask = torch.ones(B, L, device=dev)
    enc = timed(lambda: t5.generate_padded(emb, mask, 0))
    gen = timed(lambda: t5.generate_padded(emb, mask, 20))
    print(f"t5-{size} B={B} L={L}: encoder+init {enc:.3f} ms, generate20 {gen:.3f} ms, "
          f"decode {gen - enc:.3f} ms ({(gen - enc) / 20 * 1e3:.1f} us/step)", flush=True)


if __name__ == "__main__":
    main()
