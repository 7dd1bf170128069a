"""main.py-shaped harness on the GPU (BASELINE north_star: "drops into main.py unchanged").

The reference's own ``create_retrieval_dataset`` + ``predict`` + four analytics calls per batch
(main.py:119-123, 262-270) produced tests/golden/g9_main_loop.json and the cache files in
tests/golden/g9_cache/ (make_goldens.py make_g9).  Here the same calls go to a dataset object of a
reference-shaped class patched by ``dropin.patch_dataset_class`` — exactly the binding the
``python -m multimodalpromptretrieval_amd.dropin main.py ...`` launcher installs — and to the
device ``T5VisionModel`` whose retrieval function is that dataset's bound method:

* the index built over the retrieval loader matches the reference's rows (FP_TOL) and writes the
  reference's cache layout (embedding.pt / answers.pkl / answer_types.pkl);
* per test batch: predictions, retrieved answers, answer types, question info exact; the
  return_dists distances within the cdist bound;
* a second dataset object finds the reference-built cache (copied from g9_cache) and serves the
  same results without encoding anything.
"""
import json
import os
import shutil
import sys

import numpy as np
import pytest
import torch

from multimodalpromptretrieval_amd import synthetic as syn

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
sys.path.insert(0, GOLD)
import inputs as gi  # noqa: E402

FP_TOL = 2e-4


class VQASLAKEFeatureDataset:
    """Reference-shaped dataset object (the class name keys the cache directory)."""

    def __init__(self, device):
        self.device = device


def _run_main_loop(ds, model, ahead=None):
    from multimodalpromptretrieval_amd.serving import lookahead, pipelined
    out = []
    batches = gi.g9_test_batches()
    it = {None: lambda: batches, "lookahead": lambda: lookahead(batches, model),
          "serving": lambda: pipelined(batches, model)}[ahead]()
    for batch in it:
        rec = {"predictions": model.predict(batch),
               "retrieved_answers": ds.retrieve_closest_qa_pairs(batch, return_ans=True),
               "retrieved_answer_types": ds.retrieve_closest_qa_pairs(
                   batch, return_info=["question_type"]),
               "retrieved_question_info": ds.retrieve_closest_qa_pairs(
                   batch, return_info=["question", "question_id"])}
        dd = ds.retrieve_closest_qa_pairs(batch, return_dists=True)
        rec["dists_answers"] = [a for a, _ in dd]
        rec["dists"] = [[float(v) for v in d] for _, d in dd]
        out.append(rec)
    return out


def _check(got, want):
    for g, w in zip(got, want):
        for key in ("predictions", "retrieved_answers", "retrieved_answer_types",
                    "retrieved_question_info", "dists_answers"):
            assert g[key] == w[key], key
        gd, wd = np.asarray(g["dists"]), np.asarray(w["dists"])
        assert np.all(np.abs(gd ** 2 - wd ** 2) <= 2e-6 * (gd ** 2 + 2 * wd ** 2) + 1e-9)


def test_main_loop_through_dropin_binding(device, tmp_path, monkeypatch):
    from multimodalpromptretrieval_amd import dropin
    from multimodalpromptretrieval_amd.dataset import VQARetrieval, read_pickled_data
    from multimodalpromptretrieval_amd.model import T5VisionModel
    with open(os.path.join(GOLD, "g9_main_loop.json")) as f:
        want = json.load(f)["batches"]
    ccfg, clip_sd, tcfg, tok_sd, t5cfg, t5_sd = gi.g2_models()
    dropin.patch_dataset_class(VQASLAKEFeatureDataset)
    monkeypatch.chdir(tmp_path)

    ds = VQASLAKEFeatureDataset(device)
    ds._mpr_retrieval = VQARetrieval(device, clip_state_dict=clip_sd,
                                     clip_tokenizer=syn.hash_clip_tokenize)
    ds.create_retrieval_dataset(gi.g9_retrieval_loader(), "prefix", is_training_phase=False,
                                retrieval_k=gi.G9["k"])
    ref_emb = torch.load(os.path.join(GOLD, "g9_cache", "embedding.pt"), weights_only=True)
    assert ds.retrieval_embeddings.shape == ref_emb.shape
    assert float((ds.retrieval_embeddings - ref_emb).abs().max() / ref_emb.abs().max()) < FP_TOL
    mine = os.path.join(tmp_path, "cache", "VQASLAKEFeatureDataset")
    for name in ("answers.pkl", "answer_types.pkl"):
        assert read_pickled_data(os.path.join(mine, name)) == \
            read_pickled_data(os.path.join(GOLD, "g9_cache", name))
    model = T5VisionModel(device, clip_state_dict=tok_sd, t5_state_dict=t5_sd,
                          tokenizer=syn.HashT5Tokenizer(),
                          retrieval_function=ds.retrieve_closest_qa_pairs).eval()
    assert model._retrieval_obj() is ds._mpr_retrieval     # the paired tower path is taken
    _check(_run_main_loop(ds, model), want)
    # the launcher's evaluation loops (dropin.patch_dataloader): the serving loop running ahead
    # (default), and one batch ahead
    _check(_run_main_loop(ds, model, ahead="serving"), want)
    _check(_run_main_loop(ds, model, ahead="lookahead"), want)
    assert not model._hints

    # a reference-built cache is served as is (no encoding)
    shutil.rmtree(mine)
    shutil.copytree(os.path.join(GOLD, "g9_cache"), mine)
    ds2 = VQASLAKEFeatureDataset(device)
    r2 = VQARetrieval(device, clip_state_dict=clip_sd, clip_tokenizer=syn.hash_clip_tokenize)
    enc = r2.encode_queries
    r2.encode_queries = lambda b: (_ for _ in ()).throw(AssertionError("cache not used"))
    ds2._mpr_retrieval = r2
    ds2.create_retrieval_dataset(None, "prefix", is_training_phase=False, retrieval_k=gi.G9["k"])
    r2.encode_queries = enc
    assert torch.equal(ds2.retrieval_embeddings, ref_emb.float())
    model.retrieval_function = ds2.retrieve_closest_qa_pairs
    _check(_run_main_loop(ds2, model), want)
