"""Kernel trace of config C5's end-to-end leg alone (development aid): bench.c5_serving's model
over 256-question batches through the serving loop (predict_many, as the bench's pipelined
number; ``--sync``: one predict() call per batch), host sleeps around the timed window.  Run under
``rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c5t -- python tools/c5_trace.py``
then ``python tools/serving_trace.py --report gpurun_out/c5t`` (busy / idle over the window, the
longest idle gaps, kernel time by name); ``--cprofile`` adds a cProfile of one more predict()."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from multimodalpromptretrieval_amd import synthetic as syn  # noqa: E402
from multimodalpromptretrieval_amd.encoders import DeviceCLIPText  # noqa: E402
from multimodalpromptretrieval_amd.index import DeviceIndex  # noqa: E402
from multimodalpromptretrieval_amd.model import T5VisionModel  # noqa: E402
from multimodalpromptretrieval_amd.tokenization import SpmT5Tokenizer  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
n, d, B, k = bench.C5["N"], bench.C5["D"], bench.C5["B"], bench.C5["k"]
ix = DeviceIndex(syn.index_rows_device(7, 0, n, d, dev), dev)
text = DeviceCLIPText(syn.clip_state_dict(1), dev)
retr = bench._C5Retrieval(text, ix, syn.answers(n, 50), k)
m = T5VisionModel(dev, T5_version="t5-base", use_image_info=False,
                  clip_state_dict=syn.clip_state_dict(2),
                  t5_state_dict=syn.t5_state_dict(5, syn.T5_BASE),
                  tokenizer=SpmT5Tokenizer(), retrieval_function=retr).eval()
pool = bench.make_batches(int(os.environ.get("C5_BATCHES", "5")), B, seed=500, n_images=1)
os.environ["MPR_EOS_STOP_CHUNK"] = "0"
with torch.no_grad():
    for b in pool:  # every source-length bucket's graphs captured before the timed calls
        m.predict(b)
    list(m.predict_many(pool[:2], eos_stop=False))
    torch.cuda.synchronize()
    time.sleep(0.05)
    t = time.perf_counter()
    if "--sync" in sys.argv:
        parts = []
        for b in pool[1:]:
            t1 = time.perf_counter()
            m.predict(b)
            torch.cuda.synchronize()
            parts.append((time.perf_counter() - t1) * 1e3)
        print(f"{len(pool) - 1} batches: {(time.perf_counter() - t) / (len(pool) - 1) * 1e3:.2f} "
              f"ms per batch ({', '.join(f'{p:.1f}' for p in parts)})", flush=True)
    else:
        list(m.predict_many(pool[1:], eos_stop=False))
        torch.cuda.synchronize()
        print(f"{len(pool) - 1} batches through the serving loop: "
              f"{(time.perf_counter() - t) / (len(pool) - 1) * 1e3:.2f} ms per batch", flush=True)
    time.sleep(0.05)
    torch.zeros(1, device=dev).add_(1)
    torch.cuda.synchronize()
    if "--cprofile" in sys.argv:  # where the serving loop's host time goes
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        if "--sync" in sys.argv:
            m.predict(pool[1])
        else:
            list(m.predict_many(pool[1:], eos_stop=False))
        torch.cuda.synchronize()
        pr.disable()
        pstats.Stats(pr).sort_stats("cumulative").print_stats(45)
        pstats.Stats(pr).sort_stats("tottime").print_stats(25)
