"""Generate the golden fixtures under tests/golden/ from the REFERENCE ITSELF (build container only).

Run:  python tests/golden/make_goldens.py [g1 g2 g3 g4]   (needs /root/reference; never on the
GPU box — the fixtures it writes travel, the reference does not).

What is imported and executed:
* the reference's own ``VQADataset.retrieve_closest_qa_pairs`` (dataset/VQAFeatureDataset.py:187)
  called unbound on a namespace ``self`` holding a stub ``clip_model``, the index and answers;
* the reference's own ``T5VisionModel.prepare_input / predict / forward``
  (architectures/T5VisionModel.py:141-234) on an object built with ``__new__`` whose
  ``vision_model.visual``, ``T5_model`` and ``tokenizer`` are injected;
* transformers' CLIP and T5 modules as the second source for the third-party arithmetic
  (openai/CLIP is not installed; transformers 5.15.0 T5 stands in for the pinned 4.26.1).
The ``clip`` package is replaced by a stub exposing ``tokenize`` (the offline word-hash
tokenizer) — clip.load would need the network.  ``torch.argsort`` is made stable while the
reference runs, defining the order of exactly tied distances.

Weights and inputs are regenerated from numpy PCG64 seeds on both sides (tests/golden/inputs.py,
multimodalpromptretrieval_amd/synthetic.py); only reference outputs are committed.
"""
from __future__ import annotations

import json
import os
import sys
import types
from types import SimpleNamespace

import numpy as np
import torch
from torch import nn

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path[:0] = [ROOT, HERE]

from multimodalpromptretrieval_amd import synthetic as syn  # noqa: E402
import inputs as gi  # noqa: E402

# ------------------------------------------------------------------ reference import (stub clip)
clip_stub = types.ModuleType("clip")
clip_stub.tokenize = syn.hash_clip_tokenize


def _no_load(*a, **k):
    raise RuntimeError("clip.load needs the network (stubbed for golden generation)")


clip_stub.load = _no_load
sys.modules["clip"] = clip_stub
sys.path[:0] = [REF, os.path.join(REF, "dataset")]
from dataset.VQAFeatureDataset import VQADataset  # noqa: E402
from architectures.T5VisionModel import T5VisionModel  # noqa: E402

import transformers  # noqa: E402
from transformers import (CLIPTextConfig, CLIPTextModelWithProjection,  # noqa: E402
                          CLIPVisionConfig, CLIPVisionModelWithProjection)

_orig_argsort = torch.argsort


def _stable_argsort(t, dim=-1, descending=False, stable=False, **kw):
    if "axis" in kw:
        dim = kw.pop("axis")
    return _orig_argsort(t, dim=dim, descending=descending, stable=True)


torch.argsort = _stable_argsort


# ------------------------------------------------------------------ G1: retrieval scan goldens
def ref_retrieve(X, q, answers, info, k, training, **kw):
    half = X.shape[1] // 2
    clip_model = SimpleNamespace(encode_image=lambda x: q[:, :half].clone(),
                                 encode_text=lambda t: q[:, half:].clone())
    self = SimpleNamespace(clip_model=clip_model, device="cpu", retrieval_embeddings=X,
                           retrieval_answers=answers, retrieval_question_info=info,
                           retrieval_k=k, is_training_phase=training)
    batch = {"image": torch.zeros(q.shape[0], 1), "question": ["x"] * q.shape[0]}
    return VQADataset.retrieve_closest_qa_pairs(self, batch, **kw)


def make_g1():
    out = {"cases": []}
    for N, D in gi.G1_CASES:
        seed = gi.g1_seed(N, D)
        X, q, _ = gi.g1_queries(N, D, seed)
        answers = syn.answers(N, gi.G1_ANS_VOCAB)
        info = gi.question_info(N)
        for k in gi.G1_K:
            for training in (False, True):
                ids_info = ref_retrieve(X, q, answers, info, k, training,
                                        return_info=["question_id"])
                case = {
                    "N": N, "D": D, "seed": seed, "k": k, "training": training,
                    "ids": [[int(s) for s in r] for r in ids_info],
                    "prompts": ref_retrieve(X, q, answers, info, k, training),
                    "prompts_noq": ref_retrieve(X, q, answers, info, k, training,
                                                use_quantifier=False),
                    "answers": ref_retrieve(X, q, answers, info, k, training, return_ans=True),
                    "info": ref_retrieve(X, q, answers, info, k, training,
                                         return_info=["question_id", "question_type"]),
                }
                dists = ref_retrieve(X, q, answers, info, k, training, return_dists=True)
                case["dists_answers"] = [a for a, _ in dists]
                case["dists"] = [[float(v) for v in d] for _, d in dists]
                out["cases"].append(case)
    Xt, qt = gi.tie_index()
    ans = syn.answers(300, 5)
    info = gi.question_info(300)
    ties = {"cases": []}
    for k in (1, 4, 6):
        for training in (False, True):
            ties["cases"].append({
                "k": k, "training": training,
                "ids": [[int(s) for s in r] for r in
                        ref_retrieve(Xt, qt, ans, info, k, training, return_info=["question_id"])],
                "prompts": ref_retrieve(Xt, qt, ans, info, k, training)})
    out["ties"] = ties
    with open(os.path.join(HERE, "g1_retrieval.json"), "w") as f:
        json.dump(out, f)
    print("G1 cases:", len(out["cases"]), "tie cases:", len(ties["cases"]))


# ------------------------------------------------------------------ HF CLIP second source
def hf_clip_models(sd: dict, cfg: syn.ClipConfig):
    """transformers CLIP vision/text models carrying the openai-named weights in sd."""
    vc = CLIPVisionConfig(hidden_size=cfg.width, intermediate_size=4 * cfg.width,
                          num_hidden_layers=cfg.layers, num_attention_heads=cfg.heads,
                          image_size=cfg.image_size, patch_size=cfg.patch,
                          projection_dim=cfg.embed_dim, hidden_act="quick_gelu",
                          layer_norm_eps=1e-5)
    tc = CLIPTextConfig(hidden_size=cfg.text_width, intermediate_size=4 * cfg.text_width,
                        num_hidden_layers=cfg.text_layers, num_attention_heads=cfg.text_heads,
                        max_position_embeddings=cfg.context_length, vocab_size=cfg.vocab,
                        projection_dim=cfg.embed_dim, hidden_act="quick_gelu",
                        layer_norm_eps=1e-5, eos_token_id=syn.EOT, bos_token_id=syn.SOT,
                        pad_token_id=0)
    vm = CLIPVisionModelWithProjection(vc).eval()
    tm = CLIPTextModelWithProjection(tc).eval()

    def layers(prefix, hf_prefix, n, W):
        m = {}
        for i in range(n):
            p, h = f"{prefix}.resblocks.{i}", f"{hf_prefix}.encoder.layers.{i}"
            qw, kw, vw = sd[p + ".attn.in_proj_weight"].split(W)
            qb, kb, vb = sd[p + ".attn.in_proj_bias"].split(W)
            m.update({h + ".self_attn.q_proj.weight": qw, h + ".self_attn.q_proj.bias": qb,
                      h + ".self_attn.k_proj.weight": kw, h + ".self_attn.k_proj.bias": kb,
                      h + ".self_attn.v_proj.weight": vw, h + ".self_attn.v_proj.bias": vb,
                      h + ".self_attn.out_proj.weight": sd[p + ".attn.out_proj.weight"],
                      h + ".self_attn.out_proj.bias": sd[p + ".attn.out_proj.bias"],
                      h + ".layer_norm1.weight": sd[p + ".ln_1.weight"],
                      h + ".layer_norm1.bias": sd[p + ".ln_1.bias"],
                      h + ".layer_norm2.weight": sd[p + ".ln_2.weight"],
                      h + ".layer_norm2.bias": sd[p + ".ln_2.bias"],
                      h + ".mlp.fc1.weight": sd[p + ".mlp.c_fc.weight"],
                      h + ".mlp.fc1.bias": sd[p + ".mlp.c_fc.bias"],
                      h + ".mlp.fc2.weight": sd[p + ".mlp.c_proj.weight"],
                      h + ".mlp.fc2.bias": sd[p + ".mlp.c_proj.bias"]})
        return m

    v = {"vision_model.embeddings.class_embedding": sd["visual.class_embedding"],
         "vision_model.embeddings.patch_embedding.weight": sd["visual.conv1.weight"],
         "vision_model.embeddings.position_embedding.weight": sd["visual.positional_embedding"],
         "vision_model.pre_layrnorm.weight": sd["visual.ln_pre.weight"],
         "vision_model.pre_layrnorm.bias": sd["visual.ln_pre.bias"],
         "vision_model.post_layernorm.weight": sd["visual.ln_post.weight"],
         "vision_model.post_layernorm.bias": sd["visual.ln_post.bias"],
         "visual_projection.weight": sd["visual.proj"].T.contiguous()}
    v.update(layers("visual.transformer", "vision_model", cfg.layers, cfg.width))
    missing, unexpected = vm.load_state_dict(v, strict=False)
    assert not unexpected and all("position_ids" in m for m in missing), (missing, unexpected)
    t = {"text_model.embeddings.token_embedding.weight": sd["token_embedding.weight"],
         "text_model.embeddings.position_embedding.weight": sd["positional_embedding"],
         "text_model.final_layer_norm.weight": sd["ln_final.weight"],
         "text_model.final_layer_norm.bias": sd["ln_final.bias"],
         "text_projection.weight": sd["text_projection"].T.contiguous()}
    t.update(layers("transformer", "text_model", cfg.text_layers, cfg.text_width))
    missing, unexpected = tm.load_state_dict(t, strict=False)
    assert not unexpected and all("position_ids" in m for m in missing), (missing, unexpected)
    return vm, tm


@torch.no_grad()
def hf_image_tokens(vm, img):
    """embeddings -> pre_layrnorm -> encoder -> post_layernorm on ALL tokens -> projection."""
    x = vm.vision_model.embeddings(img)
    x = vm.vision_model.pre_layrnorm(x)
    x = vm.vision_model.encoder(inputs_embeds=x).last_hidden_state
    return vm.visual_projection(vm.vision_model.post_layernorm(x))


class HFVisual(nn.Module):
    """openai-CLIP-shaped ``visual`` attributes over a transformers CLIP vision model, so the
    reference's get_image_token_features (architectures/T5VisionModel.py:112-139) runs as is."""

    def __init__(self, vm):
        super().__init__()
        vis = vm.vision_model
        self.conv1 = vis.embeddings.patch_embedding
        self.class_embedding = vis.embeddings.class_embedding
        self.positional_embedding = vis.embeddings.position_embedding.weight
        self.ln_pre = vis.pre_layrnorm
        self.ln_post = vis.post_layernorm
        self.proj = vm.visual_projection.weight.T
        enc = vis.encoder
        self.transformer = lambda x: enc(inputs_embeds=x.permute(1, 0, 2)).last_hidden_state \
            .permute(1, 0, 2)


# ------------------------------------------------------------------ HF T5 second source
def hf_t5(sd: dict, cfg: syn.T5Config, dropout_rate: float = 0.0):
    tc = transformers.T5Config(d_model=cfg.d_model, d_kv=cfg.d_kv, num_heads=cfg.num_heads,
                               d_ff=cfg.d_ff, num_layers=cfg.num_layers,
                               num_decoder_layers=cfg.num_decoder_layers,
                               vocab_size=cfg.vocab_size, feed_forward_proj="relu",
                               dropout_rate=dropout_rate, decoder_start_token_id=0,
                               eos_token_id=1, pad_token_id=0, tie_word_embeddings=True)
    tc._attn_implementation = "eager"
    m = transformers.T5ForConditionalGeneration(tc).eval()
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert not unexpected and not [k for k in missing if "embed_tokens" not in k
                                   and "lm_head" not in k], (missing, unexpected)
    m.tie_weights()
    return m


# ------------------------------------------------------------------ G2: tiny end-to-end pipeline
def make_g2():
    ccfg, clip_sd, tcfg, tok_sd, t5cfg, t5_sd = gi.g2_models()
    vm_r, tm_r = hf_clip_models(clip_sd, ccfg)
    vm_t, _ = hf_clip_models(tok_sd, tcfg)
    X, answers, info = gi.g2_index(ccfg)
    with torch.no_grad():
        clip_model = SimpleNamespace(
            encode_image=lambda x: vm_r(pixel_values=x).image_embeds,
            encode_text=lambda t: tm_r(input_ids=t).text_embeds)
        rset = SimpleNamespace(clip_model=clip_model, device="cpu", retrieval_embeddings=X,
                               retrieval_answers=answers, retrieval_question_info=info,
                               retrieval_k=gi.G2["k"], is_training_phase=False)

        def retrieval_function(batch, **kw):
            return VQADataset.retrieve_closest_qa_pairs(rset, batch, **kw)

        model = T5VisionModel.__new__(T5VisionModel)
        nn.Module.__init__(model)
        model.device = "cpu"
        model.vision_encoder = "ViT-B/32"
        model.T5_version = "t5-small"
        model.max_source_length = 512
        model.max_target_length = 128
        model.use_image_info = True
        model.retrieval_function = retrieval_function
        model.use_quantifier = True
        model.use_mapping = False
        model.map_to_large = False
        model.vision_model = SimpleNamespace(visual=HFVisual(vm_t))
        model.vision_model.visual.forward = model.get_image_token_features
        tok = syn.HashT5Tokenizer()
        tok.add_tokens(["[itk]"])
        model.tokenizer = tok
        model.T5_model = hf_t5(t5_sd, t5cfg)
        model.image_token_id = tok.convert_tokens_to_ids("[itk]")
        captured = {}
        gen = model.T5_model.generate

        def gen_capture(**kw):
            out = gen(**kw)
            captured["sequences"] = out
            return out

        model.T5_model.generate = gen_capture
        batch = gi.g2_batch()
        prompts = retrieval_function(batch)
        combined, mask, enc = model.prepare_input(batch)
        preds = model.predict(batch)
        model.T5_model.generate = gen
        loss = model.forward(batch)
        model.use_quantifier = False
        prompts_noq = retrieval_function(batch, use_quantifier=False)
        combined_noq, _, enc_noq = model.prepare_input(batch)
        model.use_quantifier = True
        model.use_image_info = False
        combined_txt, mask_txt, _ = model.prepare_input(batch)
        model.use_image_info = True
        query = torch.cat([clip_model.encode_image(batch["image"]),
                           clip_model.encode_text(syn.hash_clip_tokenize(batch["question"]))], 1)
    np.savez_compressed(
        os.path.join(HERE, "g2_pipeline.npz"), combined=combined.numpy(), mask=mask.numpy(),
        input_ids=enc["input_ids"].numpy(), sequences=captured["sequences"].numpy(),
        loss=np.float32(loss.item()), combined_noq=combined_noq.numpy(),
        input_ids_noq=enc_noq["input_ids"].numpy(), combined_txt=combined_txt.numpy(),
        mask_txt=mask_txt.numpy(), query=query.numpy())
    with open(os.path.join(HERE, "g2_pipeline.json"), "w") as f:
        json.dump({"prompts": prompts, "prompts_noq": prompts_noq, "predictions": preds}, f,
                  indent=1)
    print("G2 prompts:", prompts[:2], "loss:", loss.item())


# ------------------------------------------------------------------ reference T5VisionModel shell
def ref_model(vm_t, t5_sd, t5cfg, retrieval_function, use_image_info=True, version="t5-small"):
    """The reference's T5VisionModel (architectures/T5VisionModel.py) built with __new__: its own
    prepare_input / predict / forward run; vision_model.visual, T5_model and tokenizer are
    injected (clip.load / from_pretrained need the network)."""
    model = T5VisionModel.__new__(T5VisionModel)
    nn.Module.__init__(model)
    model.device = "cpu"
    model.vision_encoder = "ViT-B/32"
    model.T5_version = version
    model.max_source_length = 512
    model.max_target_length = 128
    model.use_image_info = use_image_info
    model.retrieval_function = retrieval_function
    model.use_quantifier = True
    model.use_mapping = False
    model.map_to_large = False
    model.vision_model = SimpleNamespace(visual=HFVisual(vm_t))
    model.vision_model.visual.forward = model.get_image_token_features
    tok = syn.HashT5Tokenizer()
    tok.add_tokens(["[itk]"])
    model.tokenizer = tok
    model.T5_model = hf_t5(t5_sd, t5cfg)
    model.image_token_id = tok.convert_tokens_to_ids("[itk]")
    return model


def _g2_retrieval():
    ccfg, clip_sd, tcfg, tok_sd, t5cfg, t5_sd = gi.g2_models()
    vm_r, tm_r = hf_clip_models(clip_sd, ccfg)
    vm_t, _ = hf_clip_models(tok_sd, tcfg)
    X, answers, info = gi.g2_index(ccfg)
    clip_model = SimpleNamespace(
        encode_image=lambda x: vm_r(pixel_values=x).image_embeds,
        encode_text=lambda t: tm_r(input_ids=t).text_embeds)
    rset = SimpleNamespace(clip_model=clip_model, device="cpu", retrieval_embeddings=X,
                           retrieval_answers=answers, retrieval_question_info=info,
                           retrieval_k=gi.G2["k"], is_training_phase=False)

    def retrieval_function(batch, **kw):
        return VQADataset.retrieve_closest_qa_pairs(rset, batch, **kw)
    return vm_t, t5_sd, t5cfg, retrieval_function


def _run_model(model, batch):
    """prepare_input / predict (generate's sequences captured) / forward of the reference."""
    captured = {}
    gen = model.T5_model.generate

    def gen_capture(**kw):
        out = gen(**kw)
        captured["sequences"] = out
        return out

    model.T5_model.generate = gen_capture
    combined, mask, enc = model.prepare_input(batch)
    preds = model.predict(batch)
    model.T5_model.generate = gen
    loss = model.forward(batch)
    return combined, mask, enc, captured["sequences"], preds, loss


# ------------------------------------------------------------------ G5: utils.cosine_similarity
def make_g5():
    import utils as ref_utils  # the reference's utils.py (imported with the stub clip above)
    out = {}
    for name, x1, x2, dim in gi.g5_inputs():
        out[name] = ref_utils.cosine_similarity(x1, x2, dim=dim).numpy()
    np.savez_compressed(os.path.join(HERE, "g5_cosine.npz"), **out)
    print("G5:", {k: v.shape for k, v in out.items()})


# ------------------------------------------------------------------ G6: retrieval off (C1)
def make_g6():
    with torch.no_grad():
        vm_t, t5_sd, t5cfg, _ = _g2_retrieval()
        model = ref_model(vm_t, t5_sd, t5cfg, None)
        batch = gi.g2_batch()
        combined, mask, enc, seqs, preds, loss = _run_model(model, batch)
    np.savez_compressed(os.path.join(HERE, "g6_noretrieval.npz"), combined=combined.numpy(),
                        mask=mask.numpy(), input_ids=enc["input_ids"].numpy(),
                        sequences=seqs.numpy(), loss=np.float32(loss.item()))
    with open(os.path.join(HERE, "g6_noretrieval.json"), "w") as f:
        json.dump({"predictions": preds}, f, indent=1)
    print("G6 predictions:", preds[:2], "loss:", loss.item())


# ------------------------------------------------------------------ G7: t5-base, use_image_info=0
def make_g7():
    cfg = syn.T5_BASE
    with torch.no_grad():
        vm_t, _, _, retrieval_function = _g2_retrieval()
        t5_sd = syn.t5_state_dict(gi.G7["t5_seed"], cfg)
        model = ref_model(vm_t, t5_sd, cfg, retrieval_function, use_image_info=False,
                          version="t5-base")
        batch = gi.g2_batch()
        combined, mask, enc, seqs, preds, loss = _run_model(model, batch)
        m = model.T5_model
        emb = m.shared(enc["input_ids"])
        encd = m.encoder(inputs_embeds=emb, attention_mask=mask).last_hidden_state
        labels = seqs[:, 1:].clone()
        labels[labels == 0] = -100
        lg = m(inputs_embeds=emb, attention_mask=mask, labels=labels).logits
    sel = np.random.Generator(np.random.PCG64(gi.G7["t5_seed"] + 1)).choice(
        cfg.vocab_size, 64, replace=False)
    np.savez_compressed(os.path.join(HERE, "g7_t5_base.npz"), combined=combined.numpy(),
                        mask=mask.numpy(), input_ids=enc["input_ids"].numpy(),
                        sequences=seqs.numpy(), loss=np.float32(loss.item()),
                        enc_head=encd[:, :8].numpy(), labels=labels.numpy(),
                        logits_sel=lg[:, :, sel].numpy(), vocab_sel=sel,
                        logits_argmax=lg.argmax(-1).numpy())
    with open(os.path.join(HERE, "g7_t5_base.json"), "w") as f:
        json.dump({"predictions": preds}, f, indent=1)
    print("G7 predictions:", preds[:2], "loss:", loss.item(), "L:", mask.shape)


# ------------------------------------------------------------------ G8: long source (L = 562)
def make_g8():
    cfg = syn.T5Config()
    sd = syn.t5_state_dict(gi.G8["t5_seed"], cfg)
    m = hf_t5(sd, cfg)
    ids, img_tok, mask = gi.g8_inputs(cfg.d_model)
    with torch.no_grad():
        emb = torch.cat([img_tok, m.shared(ids)], 1)
        seqs = m.generate(inputs_embeds=emb, attention_mask=mask, do_sample=False,
                          max_new_tokens=20)
        labels = seqs[:, 1:].clone()
        labels[labels == 0] = -100
        out = m(inputs_embeds=emb, attention_mask=mask, labels=labels)
        enc = m.encoder(inputs_embeds=emb, attention_mask=mask).last_hidden_state
    sel = np.random.Generator(np.random.PCG64(gi.G8["t5_seed"] + 1)).choice(
        cfg.vocab_size, 64, replace=False)
    np.savez_compressed(os.path.join(HERE, "g8_long_source.npz"), sequences=seqs.numpy(),
                        labels=labels.numpy(), loss=np.float32(out.loss.item()),
                        logits_sel=out.logits[:, :, sel].numpy(), vocab_sel=sel,
                        logits_argmax=out.logits.argmax(-1).numpy(),
                        enc_rows=enc[:, ::37].numpy())
    print("G8 L:", emb.shape[1], "sequences:", seqs[:, :8].tolist())


# ------------------------------------------------------------------ G9: main.py-shaped harness
class VQASLAKEFeatureDataset:
    """Stands in for the reference's dataset object (its class name keys the cache directory,
    dataset/VQAFeatureDataset.py:122); the reference's own methods run on it unbound."""


def make_g9():
    import shutil
    import tempfile
    ccfg, clip_sd, tcfg, tok_sd, t5cfg, t5_sd = gi.g2_models()
    vm_r, tm_r = hf_clip_models(clip_sd, ccfg)
    vm_t, _ = hf_clip_models(tok_sd, tcfg)
    ds = VQASLAKEFeatureDataset()
    ds.device = "cpu"
    ds.clip_model = SimpleNamespace(
        encode_image=lambda x: vm_r(pixel_values=x).image_embeds,
        encode_text=lambda t: tm_r(input_ids=t).text_embeds)
    cwd = os.getcwd()
    tmp = tempfile.mkdtemp(prefix="g9_")
    out = {"batches": []}
    try:
        os.chdir(tmp)
        with torch.no_grad():
            # main.py:119-123: the index over the retrieval loader, test phase
            VQADataset.create_retrieval_dataset(ds, gi.g9_retrieval_loader(), "prefix",
                                                is_training_phase=False,
                                                retrieval_k=gi.G9["k"])

            def retrieval_function(batch, **kw):
                return VQADataset.retrieve_closest_qa_pairs(ds, batch, **kw)
            model = ref_model(vm_t, t5_sd, t5cfg, retrieval_function)
            for batch in gi.g9_test_batches():   # main.py:262-270
                rec = {"predictions": model.predict(batch),
                       "retrieved_answers": retrieval_function(batch, return_ans=True),
                       "retrieved_answer_types": retrieval_function(
                           batch, return_info=["question_type"]),
                       "retrieved_question_info": retrieval_function(
                           batch, return_info=["question", "question_id"])}
                dd = retrieval_function(batch, return_dists=True)
                rec["dists_answers"] = [a for a, _ in dd]
                rec["dists"] = [[float(v) for v in d] for _, d in dd]
                out["batches"].append(rec)
        cache = os.path.join(HERE, "g9_cache")
        shutil.rmtree(cache, ignore_errors=True)
        shutil.copytree(os.path.join(tmp, "cache", "VQASLAKEFeatureDataset"), cache)
    finally:
        os.chdir(cwd)
        shutil.rmtree(tmp, ignore_errors=True)
    with open(os.path.join(HERE, "g9_main_loop.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("G9:", out["batches"][0]["predictions"][:2], sorted(os.listdir(cache)))


# ------------------------------------------------------------------ G3 / G4: full-size second source
def make_g3():
    cfg = syn.T5Config()
    sd = syn.t5_state_dict(gi.G3["t5_seed"], cfg)
    m = hf_t5(sd, cfg)
    ids, img_tok, mask = gi.g3_inputs(cfg.d_model)
    with torch.no_grad():
        emb = torch.cat([img_tok, m.shared(ids)], 1)
        seqs = m.generate(inputs_embeds=emb, attention_mask=mask, do_sample=False,
                          max_new_tokens=20)
        labels = seqs[:, 1:].clone()
        labels[labels == 0] = -100
        out = m(inputs_embeds=emb, attention_mask=mask, labels=labels)
        enc = m.encoder(inputs_embeds=emb, attention_mask=mask).last_hidden_state
    sel = np.random.Generator(np.random.PCG64(gi.G3["vocab_sel_seed"])).choice(
        cfg.vocab_size, 64, replace=False)
    lg = out.logits
    np.savez_compressed(os.path.join(HERE, "g3_t5_small.npz"), sequences=seqs.numpy(),
                        labels=labels.numpy(), loss=np.float32(out.loss.item()),
                        logits_sel=lg[:, :, sel].numpy(), vocab_sel=sel,
                        logits_argmax=lg.argmax(-1).numpy(), logits_max=lg.max(-1).values.numpy(),
                        enc_head=enc[:, :8, :].numpy())
    print("G3 sequences:", seqs[:, :8].tolist())


def make_g4():
    cfg = syn.ClipConfig()
    sd = syn.clip_state_dict(gi.G4["clip_seed"], cfg)
    vm, tm = hf_clip_models(sd, cfg)
    img = syn.images(gi.G4["img_seed"], gi.G4["B_img"])
    toks = syn.clip_tokens(gi.G4["tok_seed"], gi.G4["B_txt"])
    with torch.no_grad():
        cls = vm(pixel_values=img).image_embeds
        tokens = hf_image_tokens(vm, img)
        txt = tm(input_ids=toks).text_embeds
    np.savez_compressed(os.path.join(HERE, "g4_clip_vit_b32.npz"), image_cls=cls.numpy(),
                        image_tokens=tokens.numpy(), text=txt.numpy())
    print("G4:", cls.shape, tokens.shape, txt.shape)


# ------------------------------------------------------------------ G10 / G11: training gradients
def _grad_record(named, rows, full=True):
    out = {}
    for n, g in named.items():
        g = g.detach()
        out["norm::" + n] = np.float64(g.double().norm().item())
        if n == "shared.weight":
            out["rows::" + n] = rows
            out["sel::" + n] = g[torch.from_numpy(rows)].numpy()
        elif full:
            out["grad::" + n] = g.numpy()
        else:
            out["head::" + n] = g.reshape(-1)[:256].numpy()
    return out


def make_g10():
    """The reference's T5VisionModel.forward (architectures/T5VisionModel.py:219-234) and
    loss.backward() (main.py:186) at G2 size: every T5 parameter gradient."""
    vm_t, t5_sd, t5cfg, retrieval_function = _g2_retrieval()
    for prm in vm_t.parameters():
        prm.requires_grad_(False)
    model = ref_model(vm_t, t5_sd, t5cfg, retrieval_function)
    batch = gi.g2_batch()
    with torch.no_grad():
        _, _, enc = model.prepare_input(batch)
        lab = model.tokenizer(batch["answer"], padding="longest", max_length=128,
                              truncation=True).input_ids
    m = model.T5_model
    m.zero_grad()
    loss = model.forward(batch)
    loss.backward()
    named = {n: p.grad for n, p in m.named_parameters() if p.grad is not None}
    rows = gi.shared_rows(gi.G10["rows_seed"], gi.G10["n_rows"], t5cfg.vocab_size,
                          list(enc["input_ids"].reshape(-1)) + [x for r in lab for x in r])
    rec = _grad_record(named, rows, full=True)
    np.savez_compressed(os.path.join(HERE, "g10_train_grads.npz"), loss=np.float32(loss.item()),
                        **rec)
    print("G10 loss:", loss.item(), "params:", len(named))


def make_g11():
    """transformers T5ForConditionalGeneration at full t5-small size: loss.backward() on the G3
    inputs (image-token rows + shared(ids), as prepare_input builds them) with G11 labels."""
    cfg = syn.T5Config()
    sd = syn.t5_state_dict(gi.G11["t5_seed"], cfg)
    m = hf_t5(sd, cfg)
    ids, img_tok, mask = gi.g3_inputs(cfg.d_model)
    labels = gi.g11_labels(ids.shape[0])
    m.zero_grad()
    emb = torch.cat([img_tok, m.shared(ids)], 1)
    loss = m(inputs_embeds=emb, attention_mask=mask, labels=labels).loss
    loss.backward()
    named = {n: p.grad for n, p in m.named_parameters() if p.grad is not None}
    rows = gi.shared_rows(gi.G11["rows_seed"], gi.G11["n_rows"], cfg.vocab_size,
                          list(ids.reshape(-1)) + [int(x) for x in labels.reshape(-1) if x >= 0])
    rec = _grad_record(named, rows, full=False)
    np.savez_compressed(os.path.join(HERE, "g11_t5_small_grads.npz"),
                        loss=np.float32(loss.item()), labels=labels.numpy(), **rec)
    print("G11 loss:", loss.item(), "params:", len(named))


class _SiteDropout(nn.Module):
    """Stands in for one of T5's nn.Dropout modules: multiplies by the counter-based mask of the
    site(s) it occupies (a T5Stack's dropout runs twice per forward: input embeddings, then the
    final-norm output)."""

    def __init__(self, seed, p, sites):
        super().__init__()
        self.seed, self.p, self.sites, self.calls = seed, p, list(sites), 0

    def forward(self, x):
        from oracle import dropout as od
        site = self.sites[self.calls]
        self.calls += 1
        return x * od.factors(self.seed, site, x.shape, self.p)


def install_site_dropout(t5, seed: int, p: float):
    """Replace every dropout of a train-mode transformers T5 by the device step's masks
    (multimodalpromptretrieval_amd/train.py dropout_site numbering).  Returns (modules, attention
    sites, a patched torch.nn.functional.dropout that takes the probability sites in call order:
    the encoder's self-attentions, then per decoder layer self then cross)."""
    from multimodalpromptretrieval_amd import train as tr
    mods = []

    def put(owner, name, sites):
        m = _SiteDropout(seed, p, sites)
        setattr(owner, name, m)
        mods.append(m)

    for stack, st in ((0, t5.encoder), (1, t5.decoder)):
        put(st, "dropout", [tr.dropout_site(stack, 255, tr.D_IN),
                            tr.dropout_site(stack, 255, tr.D_FINAL)])
        for i, blk in enumerate(st.block):
            put(blk.layer[0], "dropout", [tr.dropout_site(stack, i, tr.D_SELF_OUT)])
            if stack == 1:
                put(blk.layer[1], "dropout", [tr.dropout_site(stack, i, tr.D_CROSS_OUT)])
            ff = blk.layer[-1]
            put(ff, "dropout", [tr.dropout_site(stack, i, tr.D_FFN_OUT)])
            put(ff.DenseReluDense, "dropout", [tr.dropout_site(stack, i, tr.D_FFN_ACT)])
    asites = [tr.dropout_site(0, i, tr.D_SELF_P) for i in range(len(t5.encoder.block))]
    for i in range(len(t5.decoder.block)):
        asites += [tr.dropout_site(1, i, tr.D_SELF_P), tr.dropout_site(1, i, tr.D_CROSS_P)]
    state = {"n": 0}

    def fdropout(x, p=0.5, training=True, inplace=False, _rate=p):
        from oracle import dropout as od
        if not training or p == 0.0:
            return x
        assert abs(p - _rate) < 1e-12, p
        site = asites[state["n"]]
        state["n"] += 1
        return x * od.factors(seed, site, x.shape, _rate)
    return mods, asites, state, fdropout


def make_g12():
    """Train mode (main.py:170 model.train()): the reference's T5VisionModel.forward
    (architectures/T5VisionModel.py:219-234) + loss.backward() at G2 size with transformers' T5
    in train mode (dropout_rate 0.1) whose every dropout site is given the counter-based mask of
    the device training step (oracle/dropout.py, seed G12["seed"]): loss and every gradient."""
    vm_t, t5_sd, t5cfg, retrieval_function = _g2_retrieval()
    for prm in vm_t.parameters():
        prm.requires_grad_(False)
    model = ref_model(vm_t, t5_sd, t5cfg, retrieval_function)
    p, seed = gi.G12["p"], gi.G12["seed"]
    model.T5_model = hf_t5(t5_sd, t5cfg, dropout_rate=p)
    model.T5_model.train()
    mods, asites, state, fdropout = install_site_dropout(model.T5_model, seed, p)
    batch = gi.g2_batch()
    with torch.no_grad():
        _, _, enc = model.prepare_input(batch)
        lab = model.tokenizer(batch["answer"], padding="longest", max_length=128,
                              truncation=True).input_ids
    m = model.T5_model
    m.zero_grad()
    orig = torch.nn.functional.dropout
    torch.nn.functional.dropout = fdropout
    try:
        loss = model.forward(batch)
    finally:
        torch.nn.functional.dropout = orig
    assert state["n"] == len(asites), (state["n"], len(asites))
    assert all(md.calls == len(md.sites) for md in mods)
    loss.backward()
    named = {n: prm.grad for n, prm in m.named_parameters() if prm.grad is not None}
    rows = gi.shared_rows(gi.G10["rows_seed"], gi.G10["n_rows"], t5cfg.vocab_size,
                          list(enc["input_ids"].reshape(-1)) + [x for r in lab for x in r])
    rec = _grad_record(named, rows, full=True)
    np.savez_compressed(os.path.join(HERE, "g12_train_dropout.npz"),
                        loss=np.float32(loss.item()), p=np.float64(p), seed=np.int64(seed), **rec)
    print("G12 loss:", loss.item(), "params:", len(named))


if __name__ == "__main__":
    torch.set_num_threads(8)
    which = sys.argv[1:] or ["g1", "g2", "g3", "g4", "g5", "g6", "g7", "g8", "g9", "g10", "g11",
                             "g12"]
    for w in which:
        globals()["make_" + w]()
    with open(os.path.join(HERE, "MANIFEST.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_goldens.py", "inputs": "tests/golden/inputs.py",
                   "reference": REF, "transformers": transformers.__version__,
                   "torch": torch.__version__, "argsort": "stable=True while the reference runs",
                   "files": sorted(n for n in os.listdir(HERE) if n.startswith("g") and
                                   n not in ("g9_cache",)),
                   "g9_cache": "cache files written by the reference's create_retrieval_dataset "
                               "(dataset/VQAFeatureDataset.py:163-167)"}, f,
                  indent=1)
