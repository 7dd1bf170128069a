"""Retrieval scan timing (development aid): DeviceIndex.search at several (n, d, b, k), CUDA
events over repeated searches; reports per-search time, index GB/s and TF/s.

usage: python tools/scan_bench.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from multimodalpromptretrieval_amd.index import DeviceIndex  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(1)
    for n, d, b, k in [(6500, 1024, 16, 1), (10000, 1024, 16, 3), (8192, 1024, 16, 5),
                       (32768, 1024, 16, 5), (65536, 1024, 16, 5), (1 << 20, 512, 16, 5),
                       (1 << 20, 512, 256, 5), (1 << 17, 512, 256, 5)]:
        X = torch.randn(n, d, device=dev, generator=g) * 0.3
        q = torch.randn(b, d, device=dev, generator=g) * 0.3
        ix = DeviceIndex(X, dev)
        del X
        for _ in range(3):
            ix.search(q, k)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        it = 20
        e0.record()
        for _ in range(it):
            ix.search(q, k)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / it
        gbs = n * d * 4 / (ms * 1e-3) / 1e9
        tfs = 2.0 * n * d * b / (ms * 1e-3) / 1e12
        print(f"n={n:8d} d={d:5d} b={b:4d} k={k}: {ms * 1e3:9.1f} us  index {gbs:7.0f} GB/s  "
              f"{tfs:6.1f} TF/s", flush=True)
        del ix
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
