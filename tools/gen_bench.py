"""Generate timing (development aid): a t5-small greedy generate of one 16-row batch, of two
batches sharing one decode loop (generate_pair) and of the same two batches as two calls, alone
on the device on one stream; CUDA events over repeated calls (max_new 20, and 1 = the encoder
side alone).

usage: python tools/gen_bench.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from multimodalpromptretrieval_amd import synthetic as syn  # noqa: E402
from multimodalpromptretrieval_amd.t5 import DeviceT5  # noqa: E402


def batch(sd, b, seed, L):
    g = torch.Generator().manual_seed(seed)
    emb = torch.randn(b, L, 512, generator=g) * 0.5
    ids = torch.randint(2, 32000, (b, L - 50), generator=g)
    emb[:, 50:] = sd["shared.weight"][ids]
    return emb.cuda(), torch.ones(b, L).cuda()


def timed(fn, it=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


def main():
    sd = syn.t5_state_dict(5)
    m = DeviceT5(sd, torch.device("cuda:0"))
    a, b = batch(sd, 16, 1, 72), batch(sd, 16, 2, 72)
    for T in (20, 1):
        t1 = timed(lambda: m.generate_padded(*a, T))
        t2 = timed(lambda: m.generate_pair_padded(*a, *b, T))
        t3 = timed(lambda: (m.generate_padded(*a, T, slot=0), m.generate_padded(*b, T, slot=1)))
        print(f"max_new={T:2d}: one 16-row generate {t1 * 1e3:8.1f} us | pair 16+16 "
              f"{t2 * 1e3:8.1f} us | two 16-row generates {t3 * 1e3:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
