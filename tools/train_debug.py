"""Per-parameter gradient error of train.py against transformers T5 in float64 (development aid):
G11 inputs at full t5-small size (or G2-size with arg 'small'); prints rel errors in layer order."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "tests", "golden"))
import torch  # noqa: E402
import transformers  # noqa: E402

import inputs as gi  # noqa: E402
from multimodalpromptretrieval_amd import synthetic as syn  # noqa: E402
from multimodalpromptretrieval_amd.train import embed_rows, t5_loss  # noqa: E402

torch.set_num_threads(16)
cfg = syn.T5Config() if "small" not in sys.argv else syn.T5Config(**gi.G2["t5_cfg"])
sd = syn.t5_state_dict(gi.G11["t5_seed"], cfg)
tc = transformers.T5Config(d_model=cfg.d_model, d_kv=cfg.d_kv, num_heads=cfg.num_heads,
                           d_ff=cfg.d_ff, num_layers=cfg.num_layers,
                           num_decoder_layers=cfg.num_decoder_layers, vocab_size=cfg.vocab_size,
                           feed_forward_proj="relu", dropout_rate=0.0, decoder_start_token_id=0,
                           eos_token_id=1, pad_token_id=0, tie_word_embeddings=True)
m = transformers.T5ForConditionalGeneration(tc).eval()
m.load_state_dict(sd, strict=False)
m.tie_weights()
m = m.double()
ids, img_tok, mask = gi.g3_inputs(cfg.d_model)
labels = gi.g11_labels(ids.shape[0])
emb = torch.cat([img_tok.double(), m.shared(ids)], 1)
out = m(inputs_embeds=emb, attention_mask=mask, labels=labels)
out.loss.backward()
ref = {n: p.grad for n, p in m.named_parameters() if p.grad is not None}
dev = torch.device("cuda:0")
params = {n: torch.nn.Parameter(v.to(dev)) for n, v in sd.items()
          if n not in ("lm_head.weight", "encoder.embed_tokens.weight", "decoder.embed_tokens.weight")}
e = torch.cat([img_tok.to(dev), embed_rows(params["shared.weight"], ids)], 1)
loss = t5_loss(params, e, mask.to(dev), labels.to(dev), num_heads=cfg.num_heads)
loss.backward()
print("loss", float(loss), "ref64", float(out.loss))
for n, g in ref.items():
    a = params[n].grad.double().cpu()
    print(f"{n:70s} {float((a - g).norm() / g.norm()):.3e}")

# relu-mask agreement of every encoder/decoder FFN (our forward vs the fp64 pre-activations)
from multimodalpromptretrieval_amd import train as tr  # noqa: E402
pre = {}
for stack in ("encoder", "decoder"):
    for i, blk in enumerate(getattr(m, stack).block):
        ff = blk.layer[-1].DenseReluDense.wi
        ff.register_forward_hook(lambda mod, a, o, key=(stack, i): pre.__setitem__(key, o.detach()))
with torch.no_grad():
    m(inputs_embeds=emb, attention_mask=mask, labels=labels)
names = list(params)
order = tr.t5_param_names(tr._layers(names, "encoder"), tr._layers(names, "decoder"))
cfgt = tr.T5Config(order, {n: tuple(params[n].shape) for n in order}, cfg.num_heads)
run = tr._Runner(cfgt, [params[n] for n in order])
with torch.no_grad():
    _, tape = run.forward(e.detach(), mask.to(dev), labels.to(dev))
for stack in ("enc", "dec"):
    for i, t in enumerate(tape[stack]):
        ours = t["f"].cpu().double().reshape(-1) > 0
        ref = pre[("encoder" if stack == "enc" else "decoder", i)].reshape(-1) > 0
        bad = (ours != ref).nonzero().reshape(-1)
        vals = pre[("encoder" if stack == "enc" else "decoder", i)].reshape(-1)[bad]
        print(stack, i, "relu flips", int(bad.numel()), "ref pre-activations", vals.tolist()[:4],
              "scale", float(pre[("encoder" if stack == "enc" else "decoder", i)].abs().mean()))
