"""Greedy generation that stops where GenerationMixin stops (architectures/T5VisionModel.py:
200-205 -> greedy search ends once every row has emitted eos): mpr_t5_generate_stop runs the
decode as chunks of steps and launches no chunk after all rows finished.  Its tokens must equal
the full max_new-step loop's (the steps not run leave pad columns, which the trim cuts as
GenerationMixin's output shape does)."""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import inputs as gi  # noqa: E402

from multimodalpromptretrieval_amd import synthetic as syn  # noqa: E402
from multimodalpromptretrieval_amd.t5 import DeviceT5  # noqa: E402

pytestmark = pytest.mark.gpu


def _inputs(device, B=6, L=23, d=128, seed=11):
    g = torch.Generator().manual_seed(seed)
    emb = torch.randn((B, L, d), generator=g) * 0.5
    mask = torch.ones((B, L))
    mask[1, 17:] = 0
    mask[4, 9:] = 0
    return emb.to(device), mask.to(device)


@pytest.mark.parametrize("chunk", [2, 3, 7])
def test_generate_stop_equals_full_loop(device, monkeypatch, chunk):
    _, _, _, _, t5cfg, sd = gi.g2_models()
    dev = DeviceT5(sd, device)
    emb, mask = _inputs(device)
    full = DeviceT5.trim(dev.generate_padded(emb, mask, 20))
    monkeypatch.setenv("MPR_EOS_STOP_CHUNK", str(chunk))
    got = dev.generate(emb, mask, 20)
    assert torch.equal(got, full)
    if full.shape[1] == 21:  # some row never emitted eos: every step ran
        assert dev.last_steps_run == 20


def test_generate_stops_after_every_row_emitted_eos(device, monkeypatch):
    """Decoder layers that add nothing (o / cross-o / ffn-out zero) and an untied head whose eos
    row is the start token's embedding x 100: every row emits eos at step 1, so after chunk 0's
    flags the host launches nothing more — two chunks of 2 steps run instead of 20 steps."""
    _, _, _, _, t5cfg, sd = gi.g2_models()
    sd = {k: v.clone() for k, v in sd.items()}
    for k in list(sd):
        if k.startswith("decoder.block.") and (k.endswith("SelfAttention.o.weight")
                                              or k.endswith("EncDecAttention.o.weight")
                                              or k.endswith("DenseReluDense.wo.weight")):
            sd[k].zero_()
    head = sd["shared.weight"].clone()
    head[1] = 100.0 * sd["shared.weight"][0]
    sd["lm_head.weight"] = head
    dev = DeviceT5(sd, device)
    emb, mask = _inputs(device)
    padded = dev.generate_padded(emb, mask, 20)
    assert padded[:, 1].eq(1).all() and padded[:, 2:].eq(0).all()
    full = DeviceT5.trim(padded)
    monkeypatch.setenv("MPR_EOS_STOP_CHUNK", "2")
    got = dev.generate(emb, mask, 20)
    assert torch.equal(got, full) and got.shape[1] == 2
    assert dev.last_steps_run == 4
    monkeypatch.setenv("MPR_EOS_STOP_CHUNK", "0")
    assert torch.equal(dev.generate(emb, mask, 20), full) and dev.last_steps_run == 20
