"""cProfile of the host side of bench steps (development aid; not the bench contract).

usage: python tools/host_profile.py [--steps 10]
"""
import argparse
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    cfg = bench.CONFIGS["c2"]
    model, _, _ = bench.build(cfg, dev, None)
    batches = bench.make_batches(4, cfg["B"], dev, seed=100)
    with torch.no_grad():
        for i in range(3):
            model.predict(batches[i % 4])
        torch.cuda.synchronize()
        pr = cProfile.Profile()
        pr.enable()
        for i in range(args.steps):
            model.predict(batches[i % 4])
        torch.cuda.synchronize()
        pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(30)
    st.sort_stats("cumtime").print_stats(30)


if __name__ == "__main__":
    main()
