"""The training step's stream timeline from hipEvents, unprofiled (development aid): bench.py's
train leg (main.py:177-188 under serving.lookahead) with events around the T5 forward, the
speculative backward (its side stream), predict()'s generate, the next batch's tower pass and
the optimizer step; prints each phase's start / end relative to the step's start.
usage: python tools/train_events.py [--eos-first] [--alone]   (--eos-first: bench.eos_leg runs
before; --alone: no predict() and no loader lookahead, so the T5 forward / backward / optimizer
step run with nothing beside them)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from multimodalpromptretrieval_amd import dataset, t5, train  # noqa: E402
from multimodalpromptretrieval_amd.model import T5VisionModel  # noqa: E402
from multimodalpromptretrieval_amd.serving import lookahead  # noqa: E402
from multimodalpromptretrieval_amd.tokenization import SpmT5Tokenizer  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
cfg = bench.CONFIGS["c2"]
model0, retr, weights = bench.build(cfg, dev, None)
batches = bench.make_batches(4, cfg["B"], seed=100)
if "--eos-first" in sys.argv:
    bench.eos_leg(cfg, weights, retr, dev, batches, 20)
_, tok_sd, t5_sd, _, _ = weights
m = T5VisionModel(dev, clip_state_dict=tok_sd, t5_state_dict=t5_sd, tokenizer=SpmT5Tokenizer(),
                  retrieval_function=retr.retrieve_closest_qa_pairs, t5_dropout_rate=0.1)
opt = torch.optim.AdamW(m.parameters(), lr=1e-5)
retr.is_training_phase = True
m.train()
marks = []
on = [False]


def wrap(kind, fn):
    def inner(*a, **k):
        if not on[0]:
            return fn(*a, **k)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        out = fn(*a, **k)
        e.record()
        marks.append((kind, s, e, torch.cuda.current_stream().cuda_stream))
        return out
    return inner


dataset.encode_towers_multi = wrap("towers", dataset.encode_towers_multi)
t5.DeviceT5.generate = wrap("generate", t5.DeviceT5.generate)
train.T5LossFn._native_backward = staticmethod(wrap("backward", train.T5LossFn._native_backward))
_fwd = train.T5LossFn.forward
train.T5LossFn.forward = staticmethod(wrap("t5fwd", _fwd))
opt.step = wrap("opt", opt.step)


ALONE = "--alone" in sys.argv


def step(b):
    loss = m(b)
    if not ALONE:
        m.predict(b)
    opt.zero_grad()
    loss.backward()
    opt.step()
    return loss.item()


def run(n):
    src = (dict(b, image=b["image"].view_as(b["image"]))
           for b in (batches[i % len(batches)] for i in range(n)))
    for b in (src if ALONE else lookahead(src, m)):
        step(b)


run(4)
torch.cuda.synchronize()
on[0] = True
base = torch.cuda.Event(enable_timing=True)
base.record()
t = time.perf_counter()
n = 12
run(n)
torch.cuda.synchronize()
wall = (time.perf_counter() - t) * 1e3
on[0] = False
print(f"{n} steps: {wall / n:.2f} ms per step")
names = {}
for kind, s, e, st in marks:
    names.setdefault(st, len(names))
rows = [(base.elapsed_time(s), base.elapsed_time(e), kind, names[st]) for kind, s, e, st in marks]
rows.sort()
for a, b, kind, st in rows[:60]:
    print(f"  {kind:9s} stream {st}  {a:8.2f} - {b:8.2f}  ({b - a:6.2f})")
