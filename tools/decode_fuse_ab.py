"""A/B of the decode chain with and without the q|k|v GEMV + self-attention fusion
(MPR_DECODE_FUSE_ATTN): us per 16-row greedy step (t5-small, and t5-base), as bench.decode_chain
measures it (generate with 20 steps minus generate with 0 steps, hipEvents, best of 3), the two
forms alternated on one GPU.  usage: python tools/decode_fuse_ab.py [rounds]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodalpromptretrieval_amd import synthetic as syn  # noqa: E402
from multimodalpromptretrieval_amd.t5 import DeviceT5  # noqa: E402


def timed(dev, emb, mask, n, iters=10):
    dev.generate_padded(emb, mask, n)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        dev.generate_padded(emb, mask, n)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    device = torch.device("cuda:0")
    for name, cfg in (("t5-small", syn.T5Config()), ("t5-base", syn.T5_BASE)):
        sd = syn.t5_state_dict(3, cfg)
        g = torch.Generator().manual_seed(1)
        emb = (torch.randn((16, 71, cfg.d_model), generator=g) * 0.5).to(device)
        mask = torch.ones((16, 71), device=device)
        devs = {}
        for f in ("0", "1"):
            os.environ["MPR_DECODE_FUSE_ATTN"] = f
            devs[f] = DeviceT5(sd, device)
            devs[f].generate_padded(emb, mask, 20)
        res = {"0": [], "1": []}
        for _ in range(rounds):
            for f in ("0", "1"):
                os.environ["MPR_DECODE_FUSE_ATTN"] = f
                full = min(timed(devs[f], emb, mask, 20) for _ in range(3))
                enc = min(timed(devs[f], emb, mask, 0) for _ in range(3))
                res[f].append((full - enc) * 1e3 / 20)
        same = torch.equal(devs["0"].generate_padded(emb, mask, 20).cpu(),
                           devs["1"].generate_padded(emb, mask, 20).cpu())
        print(f"{name}: us per 16-row step  unfused {[round(x, 1) for x in res['0']]}  "
              f"fused {[round(x, 1) for x in res['1']]}  tokens equal {same}", flush=True)


if __name__ == "__main__":
    main()
