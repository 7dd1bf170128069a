"""Source lengths of config C5's prompts (development aid): per 256-question batch, the padded
length (the encoder's rows per question) against the mean real length."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from multimodalpromptretrieval_amd import synthetic as syn  # noqa: E402
from multimodalpromptretrieval_amd.encoders import DeviceCLIPText  # noqa: E402
from multimodalpromptretrieval_amd.index import DeviceIndex  # noqa: E402
from multimodalpromptretrieval_amd.model import T5VisionModel  # noqa: E402
from multimodalpromptretrieval_amd.tokenization import SpmT5Tokenizer  # noqa: E402

dev = torch.device("cuda:0")
n, d, B, k = bench.C5["N"], bench.C5["D"], bench.C5["B"], bench.C5["k"]
ix = DeviceIndex(syn.index_rows_device(7, 0, n, d, dev), dev)
text = DeviceCLIPText(syn.clip_state_dict(1), dev)
retr = bench._C5Retrieval(text, ix, syn.answers(n, 50), k)
m = T5VisionModel(dev, T5_version="t5-base", use_image_info=False,
                  clip_state_dict=syn.clip_state_dict(2),
                  t5_state_dict=syn.t5_state_dict(5, syn.T5_BASE),
                  tokenizer=SpmT5Tokenizer(), retrieval_function=retr).eval()
with torch.no_grad():
    for b in bench.make_batches(4, B, seed=500, n_images=1):
        _, mask, _ = m.prepare_input(b)
        lens = mask.sum(1).float().cpu()
        print(f"padded {mask.shape[1]}, mean {lens.mean():.1f}, min {lens.min():.0f}, "
              f"rows used {lens.sum() / mask.numel():.3f}", flush=True)
