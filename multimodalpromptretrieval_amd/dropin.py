"""Run the reference's ``main.py`` UNCHANGED with its hot path on the MI355X.

    cd <reference checkout>
    python -m multimodalpromptretrieval_amd.dropin main.py --test --config config/x.json --gpu_id 0

The launcher installs two bindings, then executes ``main.py`` as ``__main__`` (runpy):

* ``architectures.T5VisionModel.T5VisionModel`` becomes ``model.T5VisionModel`` (same constructor,
  ``prepare_input`` / ``predict`` / ``forward``, ``state_dict`` keys), so ``main.py:145`` and
  ``T5VisionModelFrozen`` (``main.py:141``) build the device model;
* ``dataset.VQAFeatureDataset.VQADataset.create_retrieval_dataset`` / ``retrieve_closest_qa_pairs``
  (called on the DATASET object at ``main.py:119-123`` and ``:267-270``) delegate to a
  ``VQARetrieval`` built from that dataset's own ``clip_model`` weights and ``clip.tokenize``:
  index and query towers in HBM, one search per batch serving the four analytics calls.  The
  index cache keeps the reference's layout (``cache/<Class>/embedding.pt | answers.pkl |
  answer_types.pkl``, dataset/VQAFeatureDataset.py:122-167), read with loaders that execute
  nothing (``weights_only=True``, a pickle reader that admits no globals), so caches the reference
  built are served and caches built here are the reference's.

Evaluation loaders over a patched dataset are iterated with the serving loop running ahead
(``serving.pipelined``): while the model is in eval mode (main.py:234), ``predict(batch)`` returns
the answers a ``ServingLoop`` over the same batches computed (towers two batches per pass, decode
groups of up to 8 batches), and the four analytics calls per batch reuse that batch's search.
Batches, their order and every result are unchanged.  ``MPR_MAIN_PIPELINE=lookahead`` iterates
one batch ahead instead (``serving.lookahead``: the next batch's towers and scan beside this
batch's decode), ``=off`` not at all.  Training loaders (the model in train mode, main.py:170)
are iterated one batch ahead (``serving.lookahead``): the next batch's retrieval towers, scan
and image tokens run beside this step's T5 forward, backward and optimizer step.

The prediction-head variants (``main.py:132-139``; SURVEY.md §2 "OUT") keep the reference's own
class: their modules are imported (binding the original base class) before the swap.
``main.py --gpu_id cpu`` (or no ``--gpu_id``) selects the reference's CPU path (main.py:58-61):
the launcher then installs nothing and the reference runs as it is — the device path never falls
back to the CPU.
"""
from __future__ import annotations

import os
import sys
import types

_INSTALLED = {}


def _retrieval_for(ds):
    """The VQARetrieval behind a patched reference dataset (built on first use from the
    dataset's clip_model weights, on its device)."""
    r = ds.__dict__.get("_mpr_retrieval")
    if r is None:
        import clip

        from .dataset import VQARetrieval, clip_package_tokenizer
        sd = {k: v.detach().float() for k, v in ds.clip_model.state_dict().items()}
        # clip.tokenize restated (tokenization.ClipBPE) on the package's own vocabulary
        r = VQARetrieval(ds.device, clip_state_dict=sd,
                         clip_tokenizer=clip_package_tokenizer() or clip.tokenize)
        ds.__dict__["_mpr_retrieval"] = r
    return r


def _create_retrieval_dataset(self, data_loader, prefix, is_training_phase=True, retrieval_k=15,
                              use_additional_data=False):
    """dataset/VQAFeatureDataset.py:118-185 on the device, reference cache layout."""
    r = _retrieval_for(self)
    r.create_retrieval_dataset(data_loader, prefix, is_training_phase=is_training_phase,
                               retrieval_k=retrieval_k, use_additional_data=use_additional_data,
                               cache_dir="cache", layout="reference",
                               cache_name=type(self).__name__)
    # the attributes the reference sets (main.py and its analytics read them)
    self.is_training_phase = is_training_phase
    self.retrieval_k = retrieval_k
    self.retrieval_embeddings = r.retrieval_embeddings
    self.retrieval_answers = r.retrieval_answers
    self.retrieval_question_info = r.retrieval_question_info
    print(f"Retrieval features shape: {tuple(self.retrieval_embeddings.shape)}")
    print(f"Number of answers: {len(self.retrieval_answers)}")


def _retrieve_closest_qa_pairs(self, batch, return_ans=False, return_info=None,
                               return_dists=False, use_quantifier=True):
    """dataset/VQAFeatureDataset.py:187-246 (same four return types)."""
    return _retrieval_for(self).retrieve_closest_qa_pairs(
        batch, return_ans=return_ans, return_info=return_info, return_dists=return_dists,
        use_quantifier=use_quantifier)


def patch_dataset_class(cls) -> None:
    """Route a VQADataset class's retrieval methods through VQARetrieval (idempotent)."""
    if getattr(cls, "_mpr_patched", False):
        return
    cls._mpr_orig = (getattr(cls, "create_retrieval_dataset", None),
                     getattr(cls, "retrieve_closest_qa_pairs", None))
    cls.create_retrieval_dataset = _create_retrieval_dataset
    cls.retrieve_closest_qa_pairs = _retrieve_closest_qa_pairs
    cls._mpr_patched = True


def patch_model_module(mod: types.ModuleType) -> None:
    """Replace ``mod.T5VisionModel`` (architectures/T5VisionModel.py) by the device model."""
    from .model import T5VisionModel
    if mod.__dict__.get("T5VisionModel") is not T5VisionModel:
        mod._mpr_orig_T5VisionModel = mod.__dict__.get("T5VisionModel")
        mod.T5VisionModel = T5VisionModel


def _eval_model():
    """The newest live device T5VisionModel in eval mode, or None."""
    from .model import LIVE_MODELS
    for m in reversed(list(LIVE_MODELS.values())):
        if not m.training:
            return m
    return None


def _train_model():
    """The newest live device T5VisionModel in training mode, or None."""
    from .model import LIVE_MODELS
    for m in reversed(list(LIVE_MODELS.values())):
        if m.training:
            return m
    return None


def patch_dataloader() -> None:
    """Iterate DataLoaders over a patched reference dataset through the serving loop
    (``serving.pipelined``; MPR_MAIN_PIPELINE=lookahead: one batch ahead, ``serving.lookahead``;
    =off: plain) while a device model is in eval mode (main.py:234 then the test loop at
    :262-270).  The batches, their order and every result are unchanged."""
    from torch.utils.data import DataLoader
    if getattr(DataLoader, "_mpr_orig_iter", None) is not None:
        return
    orig = DataLoader.__iter__

    def __iter__(self):
        it = orig(self)
        if getattr(type(self.dataset), "_mpr_patched", False):
            mode = os.environ.get("MPR_MAIN_PIPELINE", "serving")
            if mode == "off":
                return it
            from .serving import lookahead, pipelined
            m = _eval_model()
            if m is not None:
                return lookahead(it, m) if mode == "lookahead" else pipelined(it, m)
            m = _train_model()  # main.py:170-188: the next batch's retrieval beside this step
            if m is not None:
                return lookahead(it, m)
        return it

    DataLoader._mpr_orig_iter = orig
    DataLoader.__iter__ = __iter__


def install(root: str = ".") -> None:
    """Import the reference modules from ``root`` and apply both bindings (before main.py runs)."""
    if _INSTALLED:
        return
    root = os.path.abspath(root)
    for p in (root, os.path.join(root, "dataset")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import importlib
    # out-of-scope variants first: they keep the reference's own base class
    for name in ("architectures.T5VisionModelPredictionHeadBAN",
                 "architectures.T5VisionModelPredictionHead"):
        try:
            importlib.import_module(name)
        except ImportError:
            pass
    arch = importlib.import_module("architectures.T5VisionModel")
    patch_model_module(arch)
    importlib.import_module("architectures.T5VisionModelFrozen")  # subclasses the device model
    ds = importlib.import_module("dataset.VQAFeatureDataset")
    patch_dataset_class(ds.VQADataset)
    patch_dataloader()
    _INSTALLED.update(model=arch, dataset=ds)


def wants_gpu(argv) -> bool:
    """main.py:58-61: no --gpu_id or --gpu_id cpu selects the CPU."""
    gid = None
    for i, a in enumerate(argv):
        if a == "--gpu_id" and i + 1 < len(argv):
            gid = argv[i + 1]
        elif a.startswith("--gpu_id="):
            gid = a.split("=", 1)[1]
    return bool(gid) and gid != "cpu"


def main(argv=None) -> int:
    import runpy
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv:
        print(__doc__)
        return 2
    script = argv[0]
    if wants_gpu(argv[1:]):
        install(os.path.dirname(os.path.abspath(script)))
    else:
        print("[mpr dropin] main.py runs on the CPU (no --gpu_id): the reference's own path, "
              "nothing installed", file=sys.stderr)
    sys.argv = [script] + argv[1:]
    runpy.run_path(script, run_name="__main__")
    return 0


if __name__ == "__main__":
    sys.exit(main())
