"""Host time of the training step's phases (development aid): bench.py's train leg model and
main.py:177-188 step under serving.lookahead, with host timestamps around each call and one
cProfile of 3 steps sorted by own time.  usage: python tools/train_host.py"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from multimodalpromptretrieval_amd.model import T5VisionModel  # noqa: E402
from multimodalpromptretrieval_amd.serving import lookahead  # noqa: E402
from multimodalpromptretrieval_amd.tokenization import SpmT5Tokenizer  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
cfg = bench.CONFIGS["c2"]
_, retr, weights = bench.build(cfg, dev, None)
_, tok_sd, t5_sd, _, _ = weights
m = T5VisionModel(dev, clip_state_dict=tok_sd, t5_state_dict=t5_sd, tokenizer=SpmT5Tokenizer(),
                  retrieval_function=retr.retrieve_closest_qa_pairs, t5_dropout_rate=0.1)
opt = torch.optim.AdamW(m.parameters(), lr=1e-5)
retr.is_training_phase = True
m.train()
batches = bench.make_batches(4, cfg["B"], seed=11)
acc = {}


def step(b, t_loop):
    t = [t_loop, time.perf_counter()]
    loss = m(b)
    t.append(time.perf_counter())
    m.predict(b)
    t.append(time.perf_counter())
    opt.zero_grad()
    loss.backward()
    t.append(time.perf_counter())
    opt.step()
    t.append(time.perf_counter())
    v = loss.item()
    t.append(time.perf_counter())
    for k, name in enumerate(("loader", "forward", "predict", "zero+backward", "opt.step",
                              "loss.item")):
        acc[name] = acc.get(name, 0.0) + (t[k + 1] - t[k])
    return v


def run(n):
    it = lookahead([batches[i % 4] for i in range(n)], m)
    while True:
        t = time.perf_counter()
        b = next(it, None)
        if b is None:
            break
        step(b, t)


run(4)
torch.cuda.synchronize()
acc.clear()
n = 10
t0 = time.perf_counter()
run(n)
torch.cuda.synchronize()
print(f"{n} steps: {(time.perf_counter() - t0) / n * 1e3:.2f} ms per step; host ms per step by "
      "phase (call enter to return):")
for k, v in acc.items():
    print(f"  {k:14s} {v / n * 1e3:7.3f}")
pr = cProfile.Profile()
pr.enable()
run(3)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(35)
