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
    if B > 1:
        mask[1, min(17, L - 1):] = 0
    if B > 4:
        mask[4, min(9, L - 1):] = 0
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


_eos_early = syn.eos_early_t5


@pytest.mark.parametrize("n", [1, 3, 8])
@pytest.mark.parametrize("early", [False, True])
def test_generate_begin_poll_equals_full_loop(device, n, early):
    """The non-blocking grouped form (mpr_t5_generate_begin / _poll, the serving loop's): tokens
    of every batch equal the 20-step grouped loop's; with every row done at step 1 the call ends
    after the chunks launched before the first flags were read."""
    _, _, _, _, t5cfg, sd = gi.g2_models()
    dev = DeviceT5(_eos_early(sd) if early else sd, device)
    batches = [_inputs(device, B=[6, 16, 3, 9, 1, 16, 7, 5][i], L=[23, 31, 9, 40, 12, 23, 17, 8][i],
                       seed=20 + i) for i in range(n)]
    full = dev.generate_batches_padded(batches, 20, slot=1)
    outs = dev.generate_begin(batches, 20, slot=1, stop_chunk=2, ahead=2)
    polls = 0
    while True:
        done, steps = dev.generate_poll(1)
        polls += 1
        if done:
            break
        assert polls < 10_000_000
    for a, b in zip(outs, full):
        assert torch.equal(a.cpu(), b.cpu())
    if early:
        assert all(bool(t[:, 1].eq(1).all()) for t in full)
        assert steps <= 6  # at most `ahead` chunks queued past the one whose flags ended it
    # the slot is free again, and a blocking poll of a finished slot reports done
    assert dev.generate_poll(1, wait=True)[0]
    outs = dev.generate_begin(batches, 20, slot=1, stop_chunk=0)
    assert dev.generate_poll(1, wait=True) == (True, 20)
    for a, b in zip(outs, full):
        assert torch.equal(a.cpu(), b.cpu())


def test_begin_on_busy_slot_raises(device):
    _, _, _, _, t5cfg, sd = gi.g2_models()
    dev = DeviceT5(sd, device)
    b = [_inputs(device)]
    dev.generate_begin(b, 20, slot=2, stop_chunk=2, ahead=1)
    with pytest.raises(RuntimeError, match="still has a decode in flight"):
        dev.generate_begin(b, 20, slot=2, stop_chunk=2, ahead=1)
    assert dev.generate_poll(2, wait=True)[0]


def test_serving_loop_stops_early(device):
    """predict_many / serving.pipelined with an eos-early T5: every batch's answers equal
    predict()'s and the forced-20 loop's, and each generate call launches fewer steps."""
    from multimodalpromptretrieval_amd.dataset import VQARetrieval
    from multimodalpromptretrieval_amd.model import T5VisionModel
    ccfg, clip_sd, tcfg, tok_sd, t5cfg, t5_sd = gi.g2_models()
    X, answers, info = gi.g2_index(ccfg)
    retr = VQARetrieval(device, clip_state_dict=clip_sd, clip_tokenizer=syn.hash_clip_tokenize)
    retr.set_index(X, answers, info, gi.G2["k"], False)
    model = T5VisionModel(device, clip_state_dict=tok_sd, t5_state_dict=_eos_early(t5_sd),
                          tokenizer=syn.HashT5Tokenizer(),
                          retrieval_function=retr.retrieve_closest_qa_pairs).eval()
    b0 = gi.g2_batch()
    batches = []
    for i in range(11):
        b = dict(b0)
        b["image"] = syn.images(700 + i, len(b0["question"]), gi.G2["clip_cfg"]["image_size"])
        b["question"] = [q + " which" * (i * k % 4) for k, q in enumerate(b0["question"])]
        batches.append(b)
    want = [model.predict(b) for b in batches]
    assert model._device_t5().last_steps_run < 20
    forced, stopped = [], []
    assert list(model.predict_many(batches, eos_stop=False, _loop_out=forced)) == want
    for group in (1, 4, 8):
        stopped = []
        assert list(model.predict_many(batches, eos_stop=True, decode_group=group,
                                       _loop_out=stopped)) == want
        assert stopped[0].steps_run and max(stopped[0].steps_run) < 20
    assert forced[0].steps_run and min(forced[0].steps_run) == 20
