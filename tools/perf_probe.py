"""Quick per-stage GPU timing probe (development aid; not the bench contract)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from multimodalpromptretrieval_amd import synthetic as syn  # noqa: E402
from multimodalpromptretrieval_amd.encoders import CLS, TOKENS, DeviceCLIPText, DeviceViT  # noqa
from multimodalpromptretrieval_amd.index import DeviceIndex  # noqa: E402
from multimodalpromptretrieval_amd.t5 import DeviceT5  # noqa: E402


def timeit(fn, n=20, w=3):
    for _ in range(w):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


def main():
    dev = torch.device("cuda:0")
    B = 16
    sd = syn.clip_state_dict(1)
    vit = DeviceViT(sd, dev)
    txt = DeviceCLIPText(sd, dev)
    t5 = DeviceT5(syn.t5_state_dict(2), dev)
    img = syn.images(3, B).to(dev)
    tok = syn.clip_tokens(4, B)
    X = syn.index_rows(5, 6500, 1024)
    ix = DeviceIndex(X, dev)
    q = torch.randn(B, 1024, device=dev)
    emb = torch.randn(B, 71, 512, device=dev) * 0.05
    mask = torch.ones(B, 71, device=dev)
    res = {
        "vit_cls_ms": timeit(lambda: vit(img, CLS)),
        "vit_tokens_ms": timeit(lambda: vit(img, TOKENS)),
        "clip_text_ms": timeit(lambda: txt(tok)),
        "scan_k1_ms": timeit(lambda: ix.search(q, 1), n=100),
        "t5_encode_ms": timeit(lambda: t5.encode(emb, mask)),
        "t5_generate20_ms": timeit(lambda: t5.generate_padded(emb, mask, 20), n=5),
    }
    X1 = syn.index_rows(6, 1 << 20, 512)
    ix1 = DeviceIndex(X1, dev)
    q1 = torch.randn(256, 512, device=dev)
    res["scan_1M_b256_k5_ms"] = timeit(lambda: ix1.search(q1, 5), n=5)
    q2 = torch.randn(16, 512, device=dev)
    res["scan_1M_b16_k5_ms"] = timeit(lambda: ix1.search(q2, 5), n=10)
    for k, v in res.items():
        print(f"{k:24s} {v:9.3f}")


if __name__ == "__main__":
    main()
