"""GPU: the serving loop's contract with batches that do not fit one decode piece, with
consumers that stop early, and beside predict().

* a batch of more than 16 rows (a DataLoader with batch_size > 16; config C5's 256 questions)
  goes through predict_many / serving.pipelined as 16-row pieces and gets exactly predict()'s
  answers (architectures/T5VisionModel.py:196-216);
* a generator dropped mid-way leaves no decode in flight: later predict() calls and a new loop
  run (their workspace slots are free);
* a batch's greedy tokens are the same in a 128-row group, in a 256-row group and in its own
  16-row decode, at full t5-small size (one decode chain per model at every row count:
  t5.hip fold_rows).
"""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import inputs as gi  # noqa: E402

from multimodalpromptretrieval_amd import synthetic as syn  # noqa: E402

pytestmark = pytest.mark.gpu


def _model(device):
    from multimodalpromptretrieval_amd.dataset import VQARetrieval
    from multimodalpromptretrieval_amd.model import T5VisionModel
    ccfg, clip_sd, tcfg, tok_sd, t5cfg, t5_sd = gi.g2_models()
    X, answers, info = gi.g2_index(ccfg)
    retr = VQARetrieval(device, clip_state_dict=clip_sd, clip_tokenizer=syn.hash_clip_tokenize)
    retr.set_index(X, answers, info, gi.G2["k"], False)
    model = T5VisionModel(device, clip_state_dict=tok_sd, t5_state_dict=t5_sd,
                          tokenizer=syn.HashT5Tokenizer(),
                          retrieval_function=retr.retrieve_closest_qa_pairs).eval()
    return model, retr


def _batch(rows, seed):
    b0 = gi.g2_batch()
    n0 = len(b0["question"])
    qs = [b0["question"][i % n0] + " which" * (i % 5) for i in range(rows)]
    return {"image": syn.images(seed, rows, gi.G2["clip_cfg"]["image_size"]), "question": qs,
            "task": [b0["task"][i % n0] for i in range(rows)],
            "answer": [b0["answer"][i % n0] for i in range(rows)]}


@pytest.mark.parametrize("eos_stop", [True, False])
def test_predict_many_batches_over_16_rows(device, eos_stop):
    model, _ = _model(device)
    batches = [_batch(r, 500 + r) for r in (6, 24, 16, 40, 3, 130)]
    want = [model.predict(b) for b in batches]
    assert [len(w) for w in want] == [6, 24, 16, 40, 3, 130]
    assert list(model.predict_many(batches, eos_stop=eos_stop)) == want
    assert list(model.predict_many(batches, decode_group=1, eos_stop=eos_stop)) == want
    from multimodalpromptretrieval_amd.serving import pipelined
    got = []
    for b in pipelined(batches, model):
        got.append(model.predict(b))
    assert got == want


def test_dropped_loop_frees_its_slots(device):
    model, _ = _model(device)
    batches = [_batch(6, 300 + i) for i in range(12)]
    want = [model.predict(b) for b in batches]
    gen = model.predict_many(batches, decode_group=2)
    assert next(gen) == want[0]
    del gen  # calls of the other batches are in flight on the loop's slots
    import gc
    gc.collect()
    assert model.predict(batches[5]) == want[5]
    assert list(model.predict_many(batches, decode_group=2)) == want


@pytest.mark.slow
def test_t5_small_grouped_rows_equal_alone(device):
    """Full-size t5-small, eight 16-row batches: decoded as one 128-row group, as one 256-row
    group and each on its own they give bit-identical tokens (the same folded chain at every row
    count; its GEMVs sum every row alike whatever the row blocking)."""
    from multimodalpromptretrieval_amd.t5 import DeviceT5
    sd = syn.t5_state_dict(gi.G3["t5_seed"], syn.T5Config())
    dev = DeviceT5(sd, device)
    g = torch.Generator().manual_seed(3)
    ins = []
    for i in range(8):
        L = 60 + 3 * i
        emb = (torch.randn((16, L, 512), generator=g) * 0.5).to(device)
        mask = torch.ones((16, L))
        mask[i % 16, L - 7:] = 0
        ins.append((emb, mask.to(device)))
    grouped = [o.cpu() for o in dev.generate_batches_padded(ins, 20, slot=1)]
    twice = [o.cpu() for o in dev.generate_batches_padded(ins + ins, 20, slot=2)]
    for a, b, c in zip(grouped, twice[:8], twice[8:]):
        assert torch.equal(a, b) and torch.equal(a, c)
    for (e, m), gr in zip(ins, grouped):
        alone = dev.generate_padded(e, m, 20, slot=0).cpu()
        assert torch.equal(alone, gr)


@pytest.mark.parametrize("rows", [40, 130])
def test_length_ordered_pieces_equal_unsorted(device, rows):
    """t5.length_pieces: a batch of more than 16 rows decoded as length-ordered pieces, each
    trimmed to its longest row, gives every row the tokens of the unsorted, untrimmed pieces
    (t5-small at full size, right-padded masks of lengths 3 .. 60)."""
    from multimodalpromptretrieval_amd.t5 import DeviceT5
    cfg = syn.T5Config()
    m = DeviceT5(syn.t5_state_dict(3, cfg), device)
    g = torch.Generator().manual_seed(rows)
    L = 60
    emb = (torch.randn((rows, L, cfg.d_model), generator=g) * 0.3).to(device)
    lens = torch.randint(3, L + 1, (rows,), generator=g)
    lens[0] = L
    mask = (torch.arange(L)[None, :] < lens[:, None]).float().to(device)
    plain = m.generate_padded(emb, mask, 20).cpu()
    ordered = m.generate_padded(emb, mask, 20, lens=lens.tolist()).cpu()
    assert torch.equal(plain, ordered)
