"""Host logic of serving.Pipelined (no GPU): a caller that never calls predict() keeps memory
bounded (get_validation_loss, reference utils.py:78-87, iterates a wrapped loader and
only calls model(batch))."""
import torch

from multimodalpromptretrieval_amd.serving import Pipelined


class _Model:
    pass


def _batches(n):
    for i in range(n):
        yield {"image": torch.full((2, 3), float(i)), "question": [f"q{i}", f"r{i}"]}


def test_pipelined_without_predict_is_bounded():
    m = _Model()
    p = Pipelined(_batches(300), m)
    seen = 0
    peak = 0
    for b in p:
        assert float(b["image"][0, 0]) == seen  # order and content unchanged
        seen += 1
        peak = max(peak, len(p.items))
    assert seen == 300
    assert peak <= Pipelined.MAX_AHEAD + 2, peak
    assert p.gen is None  # no serving loop (no streams) without a predict()
    assert p.skipped >= 300 - Pipelined.MAX_AHEAD - 2
    # the dropped batches are no longer routed to this iterator by predict()
    assert len(m.__dict__["_pipes"]) <= Pipelined.MAX_AHEAD + 2


def test_eager_role_streams_cover_the_pipeline():
    """The serving loop's, the index build's and the trainer's role streams are all created at
    device init, in one fixed order (_lib.ensure_device), so none lands on a hardware queue chosen
    by what ran before: the tower slots (dataset.py encode:towers / encode:towers{slot}), the
    generate streams of the default two calls in flight (serving.py gen:{i}) and the trainer's
    speculative backward (train.py train:spec).  The second tower slot comes second
    (profiles/r06_stream_roles.txt)."""
    from multimodalpromptretrieval_amd import _lib
    from multimodalpromptretrieval_amd.serving import ServingOptions
    roles = _lib.PIPELINE_ROLES
    assert len(set(roles)) == len(roles)
    depth = ServingOptions.resolve().depth
    needed = {"encode:towers", "encode:towers1", "train:spec"} | {f"gen:{i}" for i in range(depth)}
    assert needed <= set(roles), needed - set(roles)
    assert roles[:2] == ("encode:towers", "encode:towers1")
