"""CPU checks of the main.py drop-in binding (multimodalpromptretrieval_amd/dropin.py) and of the
reference-cache reader (no GPU work: classes are patched, not run)."""
import io
import os
import pickle
import sys
import types

import pytest
import torch

from multimodalpromptretrieval_amd import dropin
from multimodalpromptretrieval_amd.dataset import read_pickled_data

HERE = os.path.dirname(os.path.abspath(__file__))
CACHE = os.path.join(HERE, "golden", "g9_cache")


def test_reference_cache_files_read_safely():
    """The reference's create_retrieval_dataset wrote these (make_goldens.py make_g9)."""
    emb = torch.load(os.path.join(CACHE, "embedding.pt"), map_location="cpu", weights_only=True)
    answers = read_pickled_data(os.path.join(CACHE, "answers.pkl"))
    info = read_pickled_data(os.path.join(CACHE, "answer_types.pkl"))
    assert emb.shape[0] == len(answers) == 24
    assert set(info) == {"question_type", "question_id", "question"}
    assert all(len(v) == 24 for v in info.values())


class _Evil:
    def __reduce__(self):
        return (os.getcwd, ())


def test_cache_reader_refuses_globals(tmp_path):
    p = tmp_path / "answers.pkl"
    p.write_bytes(pickle.dumps([_Evil()]))
    with pytest.raises(pickle.UnpicklingError):
        read_pickled_data(str(p))
    p.write_bytes(pickle.dumps({"a": ["x", "y"], "b": [1, 2.5]}))
    assert read_pickled_data(str(p)) == {"a": ["x", "y"], "b": [1, 2.5]}


def test_patch_dataset_class_routes_both_methods():
    class VQADataset:
        def create_retrieval_dataset(self, *a, **k):
            raise AssertionError("reference method called")

        def retrieve_closest_qa_pairs(self, *a, **k):
            raise AssertionError("reference method called")

    dropin.patch_dataset_class(VQADataset)
    dropin.patch_dataset_class(VQADataset)  # idempotent
    calls = []

    class FakeRetrieval:
        retrieval_embeddings = torch.zeros(3, 4)
        retrieval_answers = ["a", "b", "c"]
        retrieval_question_info = {"question_id": ["1", "2", "3"]}

        def create_retrieval_dataset(self, loader, prefix, **kw):
            calls.append(("create", prefix, kw))

        def retrieve_closest_qa_pairs(self, batch, **kw):
            calls.append(("retrieve", kw))
            return ["prompt"]

    ds = VQADataset()
    ds._mpr_retrieval = FakeRetrieval()
    ds.create_retrieval_dataset([], "pfx", is_training_phase=False, retrieval_k=3)
    assert calls[0][0] == "create" and calls[0][2]["layout"] == "reference"
    assert calls[0][2]["cache_name"] == "VQADataset" and ds.retrieval_k == 3
    assert ds.retrieval_answers == ["a", "b", "c"]
    assert ds.retrieve_closest_qa_pairs({}, return_info=["question_id"]) == ["prompt"]
    assert calls[1] == ("retrieve", {"return_ans": False, "return_info": ["question_id"],
                                     "return_dists": False, "use_quantifier": True})


def test_patch_model_module_and_gpu_flag():
    mod = types.ModuleType("architectures.T5VisionModel")
    mod.T5VisionModel = object
    dropin.patch_model_module(mod)
    from multimodalpromptretrieval_amd.model import T5VisionModel
    assert mod.T5VisionModel is T5VisionModel and mod._mpr_orig_T5VisionModel is object
    assert dropin.wants_gpu(["--test", "--gpu_id", "0"])
    assert dropin.wants_gpu(["--gpu_id=3"])
    assert not dropin.wants_gpu(["--test", "--gpu_id", "cpu"])
    assert not dropin.wants_gpu(["--test"])


def test_launcher_leaves_cpu_runs_to_the_reference(tmp_path, capsys):
    script = tmp_path / "main.py"
    script.write_text("import sys\nprint('ran', sys.argv[1:])\n")
    assert dropin.main([str(script), "--test", "--gpu_id", "cpu"]) == 0
    out = capsys.readouterr()
    assert "ran ['--test', '--gpu_id', 'cpu']" in out.out
    assert not dropin._INSTALLED


def test_lookahead_hints_one_batch_ahead_in_order():
    from multimodalpromptretrieval_amd.serving import lookahead
    log = []

    class FakeModel:
        training = False

        def hint_next(self, b):
            log.append(("hint", b))
            return True

    for b in lookahead(iter([1, 2, 3]), FakeModel()):
        log.append(("use", b))
    assert log == [("hint", 1), ("hint", 2), ("use", 1), ("hint", 3), ("use", 2), ("use", 3)]
    assert list(lookahead([], FakeModel())) == []


def test_pipelined_hands_out_batches_in_order_with_the_loops_answers(monkeypatch):
    """serving.pipelined: the caller gets every batch in order; a batch's answers come from the
    serving loop, pumped only as far as that batch (the loop pulls batches ahead of the caller:
    here decode groups of 3)."""
    from multimodalpromptretrieval_amd import serving
    pulled = []

    class FakeLoop:
        def __init__(self, m, o):
            pass

        def run(self, batches):
            buf = []
            for b in batches:
                pulled.append(b["id"])
                buf.append(b)
                if len(buf) == 3:
                    yield from (f"ans{x['id']}" for x in buf)
                    buf = []
            yield from (f"ans{x['id']}" for x in buf)

    monkeypatch.setattr(serving, "ServingLoop", FakeLoop)

    class M:
        training = False

    m = M()
    batches = [{"image": object(), "id": i} for i in range(7)]
    out = []
    for b in serving.pipelined(batches, m, serving.ServingOptions.resolve()):
        pipe = m._pipes.pop(id(b["image"]))
        out.append((b["id"], pipe.answers_for(b), len(pulled)))
    assert [o[:2] for o in out] == [(i, f"ans{i}") for i in range(7)]
    assert [o[2] for o in out] == [3, 3, 3, 6, 6, 6, 7]  # pumped one decode group at a time
    assert pipe.answers_for({"image": object()}) is None  # never fed: predict() runs as usual


def test_dataloader_patch_wraps_only_patched_datasets(monkeypatch):
    from torch.utils.data import DataLoader
    monkeypatch.setenv("MPR_MAIN_PIPELINE", "lookahead")

    from multimodalpromptretrieval_amd.model import LIVE_MODELS
    saved = DataLoader.__iter__
    hints = []

    class FakeModel:
        training = False

        def hint_next(self, b):
            hints.append(int(b))
            return True

    class VQADataset(torch.utils.data.Dataset):
        _mpr_patched = True

        def __len__(self):
            return 3

        def __getitem__(self, i):
            return i

    class Other(VQADataset):
        _mpr_patched = False

    fake = FakeModel()
    try:
        dropin.patch_dataloader()
        dropin.patch_dataloader()  # idempotent
        LIVE_MODELS[id(fake)] = fake
        assert [int(b) for b in DataLoader(VQADataset(), batch_size=1)] == [0, 1, 2]
        assert hints == [0, 1, 2]
        assert [int(b) for b in DataLoader(Other(), batch_size=1)] == [0, 1, 2]
        fake.training = True  # a training loop: one batch ahead whatever MPR_MAIN_PIPELINE
        monkeypatch.setenv("MPR_MAIN_PIPELINE", "serving")
        assert [int(b) for b in DataLoader(VQADataset(), batch_size=1)] == [0, 1, 2]
        assert hints == [0, 1, 2, 0, 1, 2]
        monkeypatch.setenv("MPR_MAIN_PIPELINE", "off")
        assert [int(b) for b in DataLoader(VQADataset(), batch_size=1)] == [0, 1, 2]
        assert hints == [0, 1, 2, 0, 1, 2]
    finally:
        LIVE_MODELS.pop(id(fake), None)
        DataLoader.__iter__ = saved
        del DataLoader._mpr_orig_iter
