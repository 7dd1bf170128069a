"""cProfile of the host side of bench steps (development aid; not the bench contract): the
serving loop (predict_many, forced 20 decode steps) as the headline runs it, or ``--sync`` one
predict() at a time.

usage: python tools/host_profile.py [--steps 40] [--sync]
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
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--sync", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    cfg = bench.CONFIGS["c2"]
    model, _, _ = bench.build(cfg, dev, None)
    batches = bench.make_batches(args.steps + 8, cfg["B"], seed=100)
    with torch.no_grad():
        for i in range(3):
            model.predict(batches[i % 4])
        torch.cuda.synchronize()
        for _ in model.predict_many(batches[:8], eos_stop=False):
            pass
        torch.cuda.synchronize()
        import time
        pr = cProfile.Profile()
        t0 = time.perf_counter()
        pr.enable()
        if args.sync:
            for b in batches[8:]:
                model.predict(b)
        else:
            for _ in model.predict_many(batches[8:], eos_stop=False):
                pass
        torch.cuda.synchronize()
        pr.disable()
        el = time.perf_counter() - t0
        print(f"{args.steps} steps: {el / args.steps * 1e3:.3f} ms per step (wall, under cProfile)")
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(30)
    st.sort_stats("cumtime").print_stats(30)


if __name__ == "__main__":
    main()
