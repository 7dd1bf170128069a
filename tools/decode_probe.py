"""T5 generate timing probe (development aid): eager vs graph replay, for rocprofv3 runs."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from multimodalpromptretrieval_amd import synthetic as syn  # noqa: E402
from multimodalpromptretrieval_amd.t5 import DeviceT5  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    B, L = 16, 71
    t5 = DeviceT5(syn.t5_state_dict(2), dev)
    emb = torch.randn(B, L, 512, device=dev) * 0.05
    mask = torch.ones(B, L, device=dev)
    for mode in (sys.argv[1:] or ["1", "0"]):
        os.environ["MPR_GRAPHS"] = mode
        for _ in range(3):
            t5.generate_padded(emb, mask, 20)
        torch.cuda.synchronize()
        t = time.perf_counter()
        n = 10
        for _ in range(n):
            t5.generate_padded(emb, mask, 20)
        torch.cuda.synchronize()
        print(f"graphs={mode} generate20 {(time.perf_counter() - t) / n * 1e3:.3f} ms")
        t = time.perf_counter()
        for _ in range(n):
            t5.encode(emb, mask)
        torch.cuda.synchronize()
        print(f"encode {(time.perf_counter() - t) / n * 1e3:.3f} ms")


if __name__ == "__main__":
    main()
