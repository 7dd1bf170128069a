"""Kernel trace of the training step alone (development aid): bench.py's
train leg model (t5-small + ViT-B/32 token features, batch 16, dropout 0.1) running main.py:177-188
steps (forward, predict, backward, AdamW, loss.item()) with host sleeps around the timed steps.
Run under ``rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tt -- python
tools/train_trace.py [steps]`` then ``python tools/serving_trace.py --report gpurun_out/tt``
(busy / idle over the window, the longest idle gaps, kernel time by name)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from multimodalpromptretrieval_amd.model import T5VisionModel  # noqa: E402
from multimodalpromptretrieval_amd.tokenization import SpmT5Tokenizer  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
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


def step(b):
    loss = m(b)
    m.predict(b)
    opt.zero_grad()
    loss.backward()
    opt.step()
    return loss.item()


from multimodalpromptretrieval_amd.serving import lookahead  # noqa: E402

# as the bench's train leg: the loader one batch ahead (serving.lookahead -> hint_next)
for b in lookahead([batches[i % 4] for i in range(3)], m):
    step(b)
torch.cuda.synchronize()
time.sleep(0.05)
t0 = time.perf_counter()
for b in lookahead([batches[i % 4] for i in range(steps)], m):
    step(b)
torch.cuda.synchronize()
print(f"{steps} train steps: {(time.perf_counter() - t0) / steps * 1e3:.2f} ms per step",
      flush=True)
time.sleep(0.05)
torch.zeros(1, device=dev).add_(1)
torch.cuda.synchronize()
if "--cprofile" in sys.argv:  # where one step's host time goes
    import cProfile
    import pstats
    pr = cProfile.Profile()
    pr.enable()
    for b in lookahead([batches[i % 4] for i in range(3)], m):
        step(b)
    pr.disable()
    pstats.Stats(pr).sort_stats("cumulative").print_stats(40)
