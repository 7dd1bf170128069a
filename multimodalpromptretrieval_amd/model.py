"""``T5VisionModel`` — drop-in for architectures/T5VisionModel.py on the MI355X.

Same constructor, same ``prepare_input`` / ``predict`` / ``forward`` contracts, same attributes
(``device``, ``tokenizer``, ``T5_model`` with ``shared`` / ``generate`` / ``__call__``,
``vision_model.visual`` callable) and the same ``state_dict`` keys (``vision_model.*`` in openai
CLIP naming, ``T5_model.*`` in transformers naming), so ``main.py`` and its checkpoints work
unchanged.  The arithmetic runs in libmpr: the token-feature ViT (get_image_token_features,
:112-139), the T5 embedding gather (:169), the encoder + greedy decoder (:200-205) and the
teacher-forced loss (:233).  Parameters stay the PyTorch source of truth; the device handles are
rebuilt from them whenever they change (load_state_dict, optimizer steps, .to()).

Scope notes: ``forward`` is differentiable in grad mode (train.py: the whole T5 as one autograd
node with a written-out backward; in train mode with T5's dropout at transformers' sites, rate
``t5_dropout_rate``).  ``predict()`` decodes deterministically in either mode (the reference's
train-mode predict at main.py:179 runs generate with dropout active, but its result is unused
for the generative model).  RN vision encoders, the mapping checkpoint and t5-large's untrained
512->1024 projection raise NotImplementedError; ``predict(output_attentions=True)`` (attention
plots) is out of scope.  As in the reference, image tokens (512-d) only fit a
512-d T5 (t5-small); other widths raise like the reference's torch.cat.
"""
from __future__ import annotations

import os
import weakref
from collections import deque

import torch
from torch import nn

from . import _lib
from .encoders import TOKENS, DeviceViT
from .staging import to_device
from .t5 import DeviceT5


class ParamTree(nn.Module):
    """nn.Module tree whose parameter names reproduce a flat state_dict's dotted keys."""

    def __init__(self, flat: dict = None):
        super().__init__()
        for k, v in (flat or {}).items():
            self.put(k, v)

    def put(self, key: str, value, requires_grad: bool = False):
        parts = key.split(".")
        mod = self
        for p in parts[:-1]:
            if not hasattr(mod, p) or getattr(mod, p) is None:
                mod.add_module(p, ParamTree())
            mod = getattr(mod, p)
        if isinstance(value, nn.Parameter):
            mod.register_parameter(parts[-1], value)
        else:
            mod.register_parameter(parts[-1], nn.Parameter(value.detach().clone(),
                                                           requires_grad=requires_grad))


class _VisualTower(ParamTree):
    """``vision_model.visual``: calling it returns the [B, 50, 512] token features."""

    def forward(self, x):
        return self._owner_fn(x)


class _CLIPParams(ParamTree):
    def __init__(self, sd: dict):
        super().__init__()
        self.add_module("visual", _VisualTower())
        for k, v in sd.items():
            self.put(k, v)


class _GenerationOutput:
    def __init__(self, loss, logits):
        self.loss = loss
        self.logits = logits


class T5Shell(ParamTree):
    """``T5_model``: parameters under transformers names + generate / __call__ on the device."""

    def __init__(self, sd: dict, owner, dropout_rate: float = 0.1):
        super().__init__()
        # T5Config.dropout_rate (0.1 for t5-small / t5-base): applied in train mode
        self.dropout_rate = float(dropout_rate)
        self.next_dropout_seed = None  # tests: the seed of the next train-mode forward
        # trainable like the reference's T5ForConditionalGeneration (its vision tower is frozen,
        # architectures/T5VisionModel.py:29-30); loss.backward() reaches them through train.py
        shared = nn.Parameter(sd["shared.weight"].detach().clone(), requires_grad=True)
        self.shared = nn.Embedding(shared.shape[0], shared.shape[1])
        self.shared.weight = shared
        for k, v in sd.items():
            if k in ("shared.weight", "lm_head.weight", "encoder.embed_tokens.weight",
                     "decoder.embed_tokens.weight"):
                continue
            self.put(k, v, requires_grad=True)
        # tied weights share one Parameter (T5ForConditionalGeneration tie_word_embeddings)
        self.put("encoder.embed_tokens.weight", shared)
        self.put("decoder.embed_tokens.weight", shared)
        self.put("lm_head.weight", shared)
        object.__setattr__(self, "_owner", owner)

    def generate(self, inputs_embeds=None, attention_mask=None, do_sample=False,
                 max_new_tokens=20, **kw):
        if do_sample:
            raise NotImplementedError("sampling is not on the reference's path (do_sample=False)")
        dev = self._owner._device_t5()
        return dev.generate(inputs_embeds, attention_mask, max_new_tokens).to(
            self._owner.device)

    def forward(self, inputs_embeds=None, attention_mask=None, labels=None,
                decoder_input_ids=None, **kw):
        dev = self._owner._device_t5()
        if attention_mask is None:
            attention_mask = torch.ones(inputs_embeds.shape[:2], device=inputs_embeds.device)
        if decoder_input_ids is None:
            if labels is None:
                raise ValueError("need labels or decoder_input_ids")
            decoder_input_ids = labels.new_zeros(labels.shape)
            decoder_input_ids[:, 1:] = labels[:, :-1]
            decoder_input_ids.masked_fill_(decoder_input_ids == -100, 0)
        drop = self.dropout_rate if self.training else 0.0
        if labels is not None and (drop > 0.0 or (torch.is_grad_enabled() and any(
                p.requires_grad for p in self.parameters()))):
            # differentiable loss (train.py): one autograd node over the whole T5; in train mode
            # with transformers' dropout sites (even without grad, as T5 in train mode does)
            from .train import t5_loss
            seed, self.next_dropout_seed = self.next_dropout_seed, None
            loss = t5_loss(dict(self.named_parameters()), inputs_embeds, attention_mask, labels,
                           num_heads=dev.num_heads, scale_out=dev.scale_out,
                           dropout_rate=drop, dropout_seed=seed)
            return _GenerationOutput(loss, None)
        logits = dev.logits(inputs_embeds, attention_mask, decoder_input_ids)
        loss = dev.loss(logits, labels) if labels is not None else None
        return _GenerationOutput(loss, logits)


def _load_t5(version: str, tokenizer):
    try:
        from transformers import T5ForConditionalGeneration
        m = T5ForConditionalGeneration.from_pretrained(version)
        m.resize_token_embeddings(len(tokenizer))
        return {k: v.float() for k, v in m.state_dict().items()}
    except Exception as e:  # offline image: no hub access
        raise RuntimeError(f"cannot load {version} weights ({e}); pass t5_state_dict=") from e


# live device models, newest last (dropin hands main.py's evaluation batches to the newest one in
# eval mode as lookahead hints)
LIVE_MODELS: "weakref.WeakValueDictionary[int, T5VisionModel]" = weakref.WeakValueDictionary()


class T5VisionModel(nn.Module):
    def __init__(self, device, vision_encoder="ViT-B/32", T5_version="t5-small",
                 max_source_length=512, max_target_length=128, use_image_info=True,
                 vision_checkpoint=None, mapping_checkpoint=None, retrieval_function=None,
                 use_quantifier=True, *, clip_state_dict=None, t5_state_dict=None,
                 tokenizer=None, max_new_tokens=20, t5_dropout_rate=0.1):
        super().__init__()
        self.device = torch.device(device)
        _lib.ensure_device(self.device)
        self.vision_encoder = vision_encoder
        self.T5_version = T5_version
        self.max_source_length = max_source_length
        self.max_target_length = max_target_length
        self.use_image_info = use_image_info
        self.retrieval_function = retrieval_function
        self.use_quantifier = use_quantifier
        self.max_new_tokens = max_new_tokens
        self.use_mapping = bool(mapping_checkpoint)
        if self.use_mapping:
            raise NotImplementedError("mapping_checkpoint (CrossModalMapping) is not on the "
                                      "reference's main path (main.py passes None)")
        if "ViT" not in vision_encoder:
            raise NotImplementedError(f"{vision_encoder}: only the ViT-B/32 path is built")
        if "large" in T5_version:
            raise NotImplementedError("t5-large's untrained 512->1024 projection is not built")
        if clip_state_dict is None:
            from .dataset import _default_clip
            clip_state_dict, _ = _default_clip()
        if vision_checkpoint:
            ck = torch.load(vision_checkpoint, map_location="cpu", weights_only=True)
            clip_state_dict = {k: v.float() for k, v in ck["state_dict"].items()}
        if tokenizer is None:
            # the reference's T5Tokenizer (transformers 4.26.1, SentencePiece) restated on the
            # checkpoint's spiece.model from the local Hugging Face cache (tokenization.py)
            from .tokenization import SpmT5Tokenizer
            tokenizer = SpmT5Tokenizer.from_pretrained(T5_version)
        self.tokenizer = tokenizer
        self.tokenizer.add_tokens(["[itk]"])
        if t5_state_dict is None:
            t5_state_dict = _load_t5(T5_version, self.tokenizer)
        self.vision_model = _CLIPParams({k: v.float() for k, v in clip_state_dict.items()})
        object.__setattr__(self.vision_model.visual, "_owner_fn", self.get_image_token_features)
        self.T5_model = T5Shell(t5_state_dict, self, dropout_rate=t5_dropout_rate)
        self.image_token_id = self.tokenizer.convert_tokens_to_ids("[itk]")
        self._dev = {}
        self._slots = {}
        self.to(self.device)
        LIVE_MODELS[id(self)] = self

    # ---- device handles, rebuilt when parameters change ------------------------------------------
    def _params_key(self, prefix):
        # (owner module, attribute) slots are collected once per prefix; each call re-reads the
        # slot, so re-assigned Parameters, in-place updates (_version) and new storage are all
        # seen without walking the module tree (that walk cost ~0.3 ms per call).
        slots = self._slots.get(prefix)
        if slots is None:
            slots = []
            for mname, mod in self.named_modules():
                for pname in mod._parameters:
                    full = f"{mname}.{pname}" if mname else pname
                    if full.startswith(prefix):
                        slots.append((full, mod._parameters, pname))
            self._slots[prefix] = slots
        key = []
        for full, params, pname in slots:
            p = params.get(pname)
            key.append((full, None if p is None else p.data_ptr(),
                        None if p is None else p._version))
        return tuple(key)

    def _handle(self, name, prefix, build, update=None):
        key = self._params_key(prefix)
        ent = self._dev.get(name)
        if ent is None or ent[0] != key:
            if update is not None and ent is not None:
                # an update candidate: the parameters from the cached slots (named_parameters()
                # walks the module tree, ~1 ms per optimizer step), the same traversal order,
                # tied parameters kept once under their first name as named_parameters() does
                sd, seen = {}, set()
                for full, params, pname in self._slots[prefix]:
                    p = params.get(pname)
                    if p is not None and id(p) not in seen:
                        seen.add(id(p))
                        sd[full[len(prefix):]] = p.detach()
            else:
                sd = {n[len(prefix):]: p.detach() for n, p in self.named_parameters()
                      if n.startswith(prefix)}
            shapes = tuple((n, tuple(p.shape)) for n, p in sorted(sd.items()))
            if (update is not None and ent is not None and ent[2] == shapes
                    and [k[0] for k in ent[0]] == [k[0] for k in key]):
                # same parameters, new values (an optimizer step): update in place
                ent = (key, update(ent[1], sd), shapes)
            else:
                ent = (key, build(sd), shapes)
            self._dev[name] = ent
        return ent[1]

    def _device_vit(self):
        return self._handle("vit", "vision_model.", lambda sd: DeviceViT(sd, self.device))

    def _device_t5(self):
        # named_parameters() lists the tied embedding once, as shared.weight; DeviceT5 reuses it
        # for the lm_head when lm_head.weight is absent.
        def build(sd):
            dev = DeviceT5(sd, self.device)
            if _lib.separate_decode_stream(self.device.index if self.device.index is not None
                                           else torch.cuda.current_device()):
                dev.set_decode_stream(_lib.role_stream(self.device, "decode"),
                                      slot=DeviceT5.PREDICT_SLOT)
            return dev
        return self._handle("t5", "T5_model.", build, lambda dev, sd: dev.update(sd))

    # ---- reference surface -----------------------------------------------------------------------
    def get_image_token_features(self, x):
        """architectures/T5VisionModel.py:112-139 -> [B, 50, 512] fp32 on the device."""
        return self._device_vit()(x, TOKENS)

    def _retrieval_obj(self):
        """The VQARetrieval behind ``retrieval_function``: its ``__self__``, or the one a
        reference dataset patched by ``dropin`` carries (``main.py`` passes the dataset's bound
        ``retrieve_closest_qa_pairs``, main.py:123)."""
        rf = self.retrieval_function
        owner = getattr(rf, "__self__", None)
        if owner is None and hasattr(rf, "prefetch_many"):  # a retrieval object called directly
            owner = rf
        return getattr(owner, "__dict__", {}).get("_mpr_retrieval", owner)

    @staticmethod
    def _pairable(retr, vit) -> bool:
        enc = getattr(retr, "image_encoder", None)
        return (enc is not None and enc is not vit and getattr(enc, "device", None) == vit.device
                and (enc.width, enc.patch, enc.image_size, enc.layers)
                == (vit.width, vit.patch, vit.image_size, vit.layers))

    def _prefetch(self, batches, slot: int = 0, vit=None):
        """Serving-loop lookahead: with a ``VQARetrieval`` retrieval function, enqueue the
        batches' towers (one pass over 1-2 batches; the token-feature ViT paired with the
        retrieval's when pairable), index scans and top-k copies now
        (``VQARetrieval.prefetch_many``); ``prepare_input(batch, _pre=...)`` then only waits for
        them.  A list with one entry per batch (None entries when there is nothing to
        prefetch)."""
        retr = self._retrieval_obj()
        fn = getattr(retr, "prefetch_many", None)
        if fn is None or getattr(retr, "index", None) is None:
            return [None] * len(batches)
        vit = vit if vit is not None else self._device_vit()
        other = vit if self.use_image_info and self._pairable(retr, vit) else None
        return fn(batches, other, TOKENS, slot)

    def prepare_input(self, batch, _pre=None, _handles=None):
        """architectures/T5VisionModel.py:141-184.

        The token-feature ViT does not depend on retrieval, so it is enqueued first on a side
        stream and runs on the GPU while the retrieval function encodes/scans and the host
        builds and tokenises the prompts.  With a ``VQARetrieval`` retrieval function whose
        image tower has this tower's geometry, both ViTs run as one paired pass (their
        projections share launches; results identical to separate calls)."""
        # (_handles: the device models predict() already fetched — each fetch checks every
        # parameter for updates, ~0.1 ms of host time on the GPU's critical path)
        # (the device T5 handle is only needed for the no-grad embedding gather: a training
        # forward after an optimizer step must not refresh it just for its width)
        vit = _handles[0] if _handles is not None else self._device_vit()
        d_model = self.T5_model.shared.weight.shape[1]
        if self.use_image_info and vit.out_dim != d_model:
            raise RuntimeError(f"Sizes of tensors must match: image tokens are {vit.out_dim}-d, "
                               f"{self.T5_version} d_model is {d_model} (torch.cat at "
                               f"architectures/T5VisionModel.py:176)")
        cur = torch.cuda.current_stream(self.device)
        img_tok = None
        tok_stream = None
        tok_event = None
        if self.use_image_info:
            retr = self._retrieval_obj()
            pair = getattr(retr, "encode_image_pair", None)
            if _pre is not None and _pre[0] is not None:
                img_tok, tok_event = _pre  # enqueued by _prefetch with the retrieval towers
            elif pair is not None and self._pairable(retr, vit):
                # the retrieval's encode_image and this tower see the same images: one paired
                # pass (shared launches), the retrieval picks its half up in encode_queries
                img_tok, tok_stream = pair(batch, vit, TOKENS)
            else:
                img = to_device(batch["image"], self.device)
                if not hasattr(self, "_s_tok"):
                    self._s_tok = torch.cuda.Stream(self.device)
                self._s_tok.wait_stream(cur)
                img.record_stream(self._s_tok)
                with torch.cuda.stream(self._s_tok):
                    img_tok = vit(img, TOKENS)
                tok_stream = self._s_tok
        if self.retrieval_function:
            if self.use_quantifier:
                retrieved_info = self.retrieval_function(batch)
            else:
                retrieved_info = self.retrieval_function(batch, use_quantifier=False)
        else:
            retrieved_info = ["" for _ in batch["task"]]
        task_prefixes = [f"Answer the {x} question: " for x in batch["task"]]
        B = batch["image"].shape[0]
        sentences = [task_prefixes[i] + batch["question"][i] + retrieved_info[i]
                     for i in range(len(batch["question"]))]
        encoding = self.tokenizer(sentences, padding="longest",
                                  max_length=self.max_source_length, truncation=True,
                                  return_tensors="pt")
        ids = encoding["input_ids"]
        L = ids.shape[1]
        T = vit.tokens if self.use_image_info else 0
        combined = torch.empty((B, T + L, d_model), device=self.device, dtype=torch.float32)
        if self.use_image_info:
            if tok_event is not None:
                cur.wait_event(tok_event)
            else:
                cur.wait_stream(tok_stream)
            img_tok.record_stream(cur)
            combined[:, :T].copy_(img_tok)
        shared = self.T5_model.shared.weight
        if torch.is_grad_enabled() and shared.requires_grad:
            # training: the question-token gather is an autograd node (its gradient reaches the
            # tied embedding, as T5_model.shared(ids) does at :169)
            from .train import embed_rows
            q = embed_rows(shared, ids)
            combined = torch.cat([combined[:, :T], q], 1) if T else q
        else:
            t5 = _handles[1] if _handles is not None else self._device_t5()
            t5.embed(ids, combined, row0=T)
        if self.use_image_info:
            mask = torch.ones((B, T + L), dtype=torch.float32)
            mask[:, T:] = encoding["attention_mask"].float()
        else:
            mask = encoding["attention_mask"]
        return combined, _lib.to_device_async(mask, self.device), encoding

    def predict(self, batch, output_attentions=False):
        """architectures/T5VisionModel.py:196-216 (greedy, max_new_tokens=20).  A batch
        announced by ``hint_next`` picks up its already-enqueued retrieval work."""
        if output_attentions:
            raise NotImplementedError("output_attentions is the eval-only plotting path")
        pipe = self.__dict__.get("_pipes", {}).pop(id(batch["image"]), None)
        if pipe is not None:  # handed out by serving.pipelined: its loop computed the answers
            ans = pipe.answers_for(batch)
            if ans is not None:
                return ans
        memo = self._take_forward_inputs(batch)
        pre = self._take_hint(batch) if memo is None else None
        if pre is not None or memo is not None:
            # the retrieval stream may already hold the NEXT hinted batch's towers (and, after a
            # training forward, its speculative backward runs beside): the T5 part runs on a
            # stream of its own (the serving loop's first generate stream) instead of queueing
            # behind them (main.py:177-179's predict after forward: profiles/r05_train_streams.txt)
            which = os.environ.get("MPR_AHEAD_T5_STREAM", "gen:0")
            if which == "private":
                if not hasattr(self, "_s_main"):
                    self._s_main = torch.cuda.Stream(self.device)
                s_main = self._s_main
            elif which == "current":
                s_main = torch.cuda.current_stream(self.device)
            else:
                s_main = _lib.role_stream(self.device, which)
        else:
            # Whole predict() on one non-default stream: eager launches on the legacy default
            # stream cost more per kernel; the result is host strings, so no stream handoff.
            # With a VQARetrieval on this device that stream is the retrieval's own tower stream,
            # so the towers -> scan -> T5 chain has no cross-stream waits (a private stream
            # measured 10.8-13.4 ms per predict() depending on how the process's earlier streams
            # happened to map onto the 4 hardware queues; MPR_PREDICT_STREAM=private restores it).
            s_main = self._predict_stream()
        # the handles first: a T5 refreshed after an optimizer step enqueues its weight update
        # on the current stream, which s_main then waits for
        handles = (self._device_vit(), self._device_t5())
        s_main.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s_main), torch.no_grad():
            if memo is not None:
                combined, mask, lens = memo
            else:
                combined, mask, enc = self.prepare_input(batch, _pre=pre, _handles=handles)
                lens = self.row_lengths(combined, enc)
            # T5_model.generate (:200-205) hands back a device tensor as GenerationMixin does;
            # the answers only need the host copy the device generate already made, so decode
            # that one (batch_decode over a device tensor pays a D2H copy + sync per row)
            seqs = handles[1].generate(combined, mask, self.max_new_tokens, lens=lens,
                                       while_running=self._flush_hints)
        return self.tokenizer.batch_decode(seqs, skip_special_tokens=True)

    # ---- lookahead for batch-after-batch callers (main.py:262-263) ---------------------------
    MAX_HINTS = 4

    def hint_next(self, batch) -> bool:
        """Announce a batch the caller will ``predict()`` soon (``serving.lookahead`` does this
        one batch ahead; ``dropin`` wraps main.py's evaluation loaders with it).  The batch's
        device-side retrieval work — the query towers paired with the token-feature ViT, the
        index scan and the top-k copy to host (``_prefetch``) — runs on the retrieval stream
        beside the current ``predict()``'s T5 encoder and greedy decode, which leave most of the
        chip idle; the hinted ``predict()`` then only waits for it.  Same launches, same results
        as an unhinted call.  In training mode the hinted ``forward(batch)`` picks it up the same
        way (main.py:177-178: the towers are frozen and the index fixed while the T5 trains, so
        the next batch's retrieval and image tokens run beside this step's T5 forward /
        backward).

        The work is queued here and enqueued at the model's next long stretch of GPU work — a
        training forward's T5 launch, a ``predict()``'s decode (``_flush_hints``) — or when the
        batch itself is needed: a loop calls this right after the previous step's host sync,
        with the GPU idle, and staging the batch's pageable images into pinned memory (~1 ms of
        host copy) in front of the GPU work left the GPU waiting for it.  The queued work is
        ordered after what the caller's stream held at this call (an event), not after the T5
        work enqueued since.  Returns whether the batch was queued: not without a
        ``VQARetrieval`` with an index on this device, nor for a batch already hinted."""
        if not hasattr(self, "_hints"):
            self._hints = {}
            self._pending_hints = deque()
        key = id(batch["image"])
        if key in self._hints or any(b["image"] is batch["image"]
                                     for b, _ in self._pending_hints):
            return False
        retr = self._retrieval_obj()
        if (getattr(retr, "prefetch_many", None) is None or getattr(retr, "index", None) is None
                or self.device.type != "cuda"):
            return False
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self._pending_hints.append((batch, ev))
        while len(self._pending_hints) > self.MAX_HINTS:  # announced, never used: drop oldest
            self._pending_hints.popleft()
        return True

    def _flush_hints(self, upto=None):
        """Enqueue the queued hints' retrieval work (all of them, or up to and including the
        batch ``upto``) on the hint stream, each after the event its ``hint_next`` recorded."""
        pend = getattr(self, "_pending_hints", None)
        if not pend:
            return
        if not hasattr(self, "_s_hint"):
            self._s_hint = torch.cuda.Stream(self.device)
        slot = int(os.environ.get("MPR_AHEAD_SLOT", "0"))
        while pend:
            batch, ev = pend.popleft()
            self._s_hint.wait_event(ev)
            with torch.cuda.stream(self._s_hint):
                pre = self._prefetch([batch], slot)[0]
            if pre is not None:
                while len(self._hints) >= self.MAX_HINTS:  # never predicted: drop oldest
                    self._hints.pop(next(iter(self._hints)))
                # the entry holds the batch's image tensor: its id() is not reused while it lives
                self._hints[id(batch["image"])] = (batch["image"], tuple(batch["question"]), pre)
            if upto is not None and batch["image"] is upto["image"]:
                break

    def _take_hint(self, batch):
        pend = getattr(self, "_pending_hints", None)
        if pend and any(b["image"] is batch["image"] for b, _ in pend):
            self._flush_hints(upto=batch)
        hints = getattr(self, "_hints", None)
        if not hints:
            return None
        ent = hints.pop(id(batch["image"]), None)
        if ent is None or ent[0] is not batch["image"] or ent[1] != tuple(batch["question"]):
            return None
        return ent[2]

    def _predict_stream(self):
        retr = self._retrieval_obj()
        streams = getattr(retr, "_streams", None)
        if (streams is not None and getattr(retr, "device", None) == self.device
                and os.environ.get("MPR_PREDICT_STREAM", "") != "private"):
            return streams()
        if not hasattr(self, "_s_main"):
            self._s_main = torch.cuda.Stream(self.device)
        return self._s_main

    def predict_many(self, batches, decodes_in_flight: int = 2, pair_decodes=None,
                     lookahead=None, tower_slots=None, decode_group=None, tower_batches=None,
                     eos_stop=None, _loop_out=None):
        """predict() over an iterable of batches as a serving pipeline.  A greedy decode is a
        chain of small latency-bound launches that leaves most of the chip idle, so
        (1) ``decode_group`` (1-16, default MPR_DECODE_GROUP or 12; ``pair_decodes`` = False / True
        is 1 / 2) consecutive batches share one decode loop: each is encoded as predict() would,
        then their rows step together, reading every decode weight once per step for all
        (mpr_t5_generate_batches);
        (2) up to ``decodes_in_flight`` of those generate calls run at once, each on its own
        stream and T5 workspace slot, while the next batches' image towers, question tower and
        index scan run beside them and the host builds its prompts;
        (3) with ``lookahead`` (default on; MPR_LOOKAHEAD=0 turns it off) the next tower pass,
        its scans and top-k copies are enqueued before the host blocks on a retrieval result, so
        the towers never wait on the host; ``tower_batches`` (1-2, default MPR_TOWER_BATCHES or
        2) batches share one tower pass (the ViTs over their images concatenated: fewer, fuller
        launches); ``tower_slots`` > 1 (MPR_TOWER_SLOTS, default 1) overlaps consecutive passes
        on workspace slots of their own (measured slower beside the decodes).
        (4) ``eos_stop`` (default on, MPR_SERVING_EOS_STOP=0 turns it off) ends each call's
        decode at the first chunk of MPR_EOS_STOP_CHUNK steps after which every row has emitted
        eos, as greedy search stops (architectures/T5VisionModel.py:200-205), polled without
        blocking the host; off, every call runs max_new_tokens steps.
        Yields each batch's answers in order; every batch gets exactly predict()'s answers (one
        decode chain per model at every row count, whatever else shares the chip:
        serving.ServingLoop).  ``_loop_out`` (a list) receives the ServingLoop."""
        from .serving import ServingLoop, ServingOptions
        opts = ServingOptions.resolve(decodes_in_flight, pair_decodes, lookahead, tower_slots,
                                      decode_group, tower_batches, eos_stop)
        loop = ServingLoop(self, opts)
        if _loop_out is not None:
            _loop_out.append(loop)
        return loop.run(batches)

    def _finish(self, host_tokens, done):
        done.synchronize()  # this batch's tokens only; the next batch keeps running
        seqs = DeviceT5.trim(host_tokens)
        return self.tokenizer.batch_decode(seqs, skip_special_tokens=True)

    def forward(self, batch):
        """architectures/T5VisionModel.py:219-234: the teacher-forced loss; differentiable when
        grad mode is on and T5 parameters require grad (train.py), else the value only.
        The labels stay on the host (T5Shell and train.py take host or device labels; the
        reference's ``.to(device)`` copy then a ``.cpu()`` read back would wait for the GPU).
        main.py:177-179 follows ``model(batch)`` with ``model.predict(batch)`` on the same batch
        before any optimizer step: the inputs built here (retrieval, prompts, image tokens,
        question embeddings) are kept for that predict(), which would rebuild the same values."""
        combined, mask, enc = self.prepare_input(batch, _pre=self._take_hint(batch))
        self._fwd_inputs = (self._forward_key(batch), combined.detach(), mask,
                            self.row_lengths(combined, enc))
        target = self.tokenizer(batch["answer"], padding="longest",
                                max_length=self.max_target_length, truncation=True)
        labels = torch.tensor(target["input_ids"])
        labels[labels == self.tokenizer.pad_token_id] = -100
        loss = self.T5_model(inputs_embeds=combined, attention_mask=mask, labels=labels).loss
        self._flush_hints()  # the next batch's retrieval, beside this T5 forward (hint_next)
        return loss

    def _forward_key(self, batch):
        # what prepare_input's result depends on besides the batch: the tied embedding's values
        # (its in-place version: an optimizer step changes it) and the retrieval phase
        retr = self._retrieval_obj()
        return (batch["image"], tuple(batch["question"]), tuple(batch["task"]),
                self.T5_model.shared.weight._version, getattr(retr, "is_training_phase", None),
                self.use_image_info, self.use_quantifier)

    def _take_forward_inputs(self, batch):
        ent = self.__dict__.pop("_fwd_inputs", None)
        if ent is None:
            return None
        key = self._forward_key(batch)
        if ent[0][0] is not key[0] or ent[0][1:] != key[1:]:
            return None
        return ent[1], ent[2], ent[3]

    @staticmethod
    def row_lengths(combined, encoding):
        """Real length of each row of prepare_input's output (host ints, no device read): the
        image tokens plus the prompt's tokens (the tokenizer pads on the right)."""
        am = encoding["attention_mask"]
        am = am if isinstance(am, torch.Tensor) else torch.as_tensor(am)
        T = combined.shape[1] - am.shape[1]
        return (am.sum(1) + T).tolist()
