"""Host tokenizers against transformers' tokenizers on the same
vocabulary files (CPU only).

* CLIP: ``tokenization.ClipBPE`` (openai ``clip.tokenize``, dataset/VQAFeatureDataset.py:190)
  against transformers' ``CLIPTokenizer`` built from the same merges.  transformers does not
  run openai's ``basic_clean`` (ftfy + double HTML unescape), so both sides get the text after
  ``tokenization.clean``; the clean-up rules are pinned separately below.
* T5: ``tokenization.SpmT5Tokenizer`` (transformers 4.26.1's SentencePiece ``T5Tokenizer``, the
  reference's pin, requirements.txt:9) against the installed transformers ``T5Tokenizer`` (5.x,
  converted from the same ``spiece.model``) with ``[itk]`` added, ``padding="longest"``,
  ``max_length=512``, ``truncation=True`` (architectures/T5VisionModel.py:57-61,161-167).  The one
  rule where the versions differ: text ending in a literal ``</s>`` gets no second EOS in 4.26.1
  (``_add_eos_if_not_present``), which 5.x appends; those rows are checked against the 4.26.1
  rule instead.

Against openai CLIP's own vocabulary and t5-small's ``spiece.model``: parity unpinned (neither is
available offline; the vocabularies here are same-format stand-ins, vocab/make_vocab.py).
"""
import os
import warnings

import numpy as np
import pytest
import torch

from multimodalpromptretrieval_amd import tokenization as tk

WORDS = ("what is the organ shown in this image does picture contain lung liver brain which "
         "modality used where mass abnormal left right heart kidney chest abdomen ct mri x-ray "
         "largest normal spleen pancreas effusion nodule pneumothorax cardiomegaly T1 T2 "
         "weighted axial coronal sagittal plane how many are there located bigger smaller "
         "diseases included part of body belong to is it healthy color size quantity position "
         "abnormality answer question believe likely certainly maybe unlikely").split()
EXTRA = ["don't", "it's", "they're", "we've", "I'm", "you'll", "he'd", "O'Neil", "3.5cm",
         "12", "2023-10-17", "x2", "(left)", "[right]", "{a}", "#1", "50%", "a/b", "e.g.",
         "naïve", "café", "Größe", "μm", "Δx", "日本語", "лёгкое", "😀", "👍🏽", "â€™", "ﬁbrosis",
         "“quoted”", "‘single’", "ＦＵＬＬ", "&amp;", "&lt;b&gt;", "&amp;amp;", " nbsp",
         "tab\there", "new\nline", "  spaced  ", "UPPER", "MiXeD", "...", "?!", "--", "''",
         "'s", "''s", "'''", "<|endoftext|>", "<|startoftext|>", "`code`", "a_b", "1,000",
         "e=mc^2", "C++", "@user", "\x00ctrl", "\r\nwin", " sep"]


def _strings(n, seed=88):
    rng = np.random.Generator(np.random.PCG64(seed))
    out = []
    for i in range(n):
        m = int(rng.integers(1, 25))
        toks = []
        for _ in range(m):
            r = rng.random()
            if r < 0.7:
                w = WORDS[int(rng.integers(len(WORDS)))]
                c = rng.random()
                w = w.capitalize() if c < 0.15 else (w.upper() if c < 0.2 else w)
            else:
                w = EXTRA[int(rng.integers(len(EXTRA)))]
            toks.append(w)
        seps = [" ", " ", " ", "  ", "", ", ", "? ", ". "]
        s = toks[0]
        for t in toks[1:]:
            s += seps[int(rng.integers(len(seps)))] + t
        if rng.random() < 0.3:
            s += "?"
        out.append(s)
    return out


STRINGS = _strings(1200)


@pytest.fixture(scope="module")
def clip_pair():
    from transformers import CLIPTokenizer
    ours = tk.ClipBPE()
    merges = sorted(ours.ranks, key=ours.ranks.get)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        hf = CLIPTokenizer(vocab=dict(ours.encoder), merges=[tuple(m) for m in merges])
    return ours, hf


@pytest.fixture(scope="module")
def t5_pair(tmp_path_factory):
    from transformers import T5Tokenizer
    d = tmp_path_factory.mktemp("t5tok")
    os.symlink(tk.T5_SPM_DEFAULT, d / "spiece.model")
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        hf = T5Tokenizer.from_pretrained(str(d))
    hf.add_tokens(["[itk]"])
    ours = tk.SpmT5Tokenizer()
    ours.add_tokens(["[itk]"])
    return ours, hf


def test_clip_vocab_layout(clip_pair):
    ours, _ = clip_pair
    assert ours.vocab_size == 49408
    assert (ours.sot, ours.eot) == (49406, 49407)  # the real vocabulary's ids
    assert ours.encoder["!"] == 0 and ours.encoder["!</w>"] == 256


def test_clip_bpe_matches_transformers(clip_pair):
    ours, hf = clip_pair
    n = 0
    for s in STRINGS:
        if "<|" in s:  # transformers cuts its special tokens out first (below)
            continue
        c = tk.clean(s)
        a = ours.encode_cleaned(c)
        b = hf(c, add_special_tokens=False)["input_ids"]
        assert a == b, (s, c, a, b)
        assert ours.encode(s) == a  # the per-word memo path
        n += 1
    assert n >= 1000


def test_clip_special_token_literals(clip_pair):
    """openai applies its pattern left to right: a special-token literal is one piece only when
    the pattern reaches it at its '<' (transformers splits added tokens out before the pattern,
    so it differs exactly when punctuation runs into the literal)."""
    ours, hf = clip_pair
    assert ours.pat.findall("c++<|endoftext|>heart") == ["c", "++<|", "endoftext", "|>", "heart"]
    assert ours.encode("lung <|endoftext|> liver")[1] == ours.eot
    c = "lung <|startoftext|> liver"
    assert ours.encode_cleaned(c) == hf(c, add_special_tokens=False)["input_ids"]


def test_clip_tokenize_contract(clip_pair):
    ours, _ = clip_pair
    t = tk.clip_tokenize(["what is the organ?", "liver"])
    assert t.dtype == torch.int32 and t.shape == (2, 77)
    for row, s in zip(t, ["what is the organ?", "liver"]):
        ids = [ours.sot] + ours.encode(s) + [ours.eot]
        assert row[:len(ids)].tolist() == ids and not row[len(ids):].any()
        assert int(row.argmax()) == len(ids) - 1  # EOT is the largest id (encode_text's pooling)
    long = " ".join(["lung"] * 80)
    with pytest.raises(RuntimeError, match="too long for context length 77"):
        tk.clip_tokenize([long])
    tr = tk.clip_tokenize([long], truncate=True)
    assert tr.shape == (1, 77) and int(tr[0, -1]) == ours.eot and int(tr[0, 0]) == ours.sot
    assert ours.decode(ours.encode("What is the ORGAN shown?")) == "what is the organ shown ? "


def test_clip_clean_rules():
    # openai basic_clean (ftfy subset + html.unescape twice) + whitespace_clean + lower
    assert tk.clean("  Hello\t\nWorld  ") == "hello world"
    assert tk.clean("Tom &amp;amp; Jerry") == "tom & jerry"
    assert tk.clean("&lt;b&gt;") == "<b>"
    assert tk.clean("“quoted” ‘x’") == "\"quoted\" 'x'"
    assert tk.clean("ﬁbrosis") == "fibrosis"
    assert tk.clean("ＦＵＬＬ width") == "full width"
    assert tk.clean("a\x00b\x7fc") == "abc"
    assert tk.clean("café") == "café"  # NFC
    assert tk.clean("\x1b[31mred\x1b[0m") == "red"


def _rows(enc):
    return [list(r) for r in enc["input_ids"]], [list(r) for r in enc["attention_mask"]]


def test_t5_encode_matches_transformers(t5_pair):
    ours, hf = t5_pair
    assert len(ours) == len(hf) == 32101
    assert ours.convert_tokens_to_ids("[itk]") == hf.convert_tokens_to_ids("[itk]") == 32100
    prompts = [f"Answer the {t} question: {s}" for t, s in
               zip(["organ", "modality", "position", "abnormality"] * 400, STRINGS)]
    specials = ["lung <extra_id_3> liver", "a [itk] b", "<pad> x", "x <unk>", "[itk][itk]",
                "<extra_id_99>y", "hi </s> there"]
    texts = prompts + specials
    n = 0
    for i in range(0, len(texts), 16):
        batch = texts[i:i + 16]
        a = ours(batch, padding="longest", max_length=512, truncation=True)
        b = hf(batch, padding="longest", max_length=512, truncation=True)
        assert _rows(a) == _rows(b), batch
        n += len(batch)
    assert n >= 1000
    # tensors, as prepare_input asks for them
    a = ours(prompts[:16], padding="longest", max_length=512, truncation=True,
             return_tensors="pt")
    assert a["input_ids"].dtype == torch.long and a["attention_mask"].shape == a["input_ids"].shape


def test_t5_word_memo_is_whole_text_encode(t5_pair):
    ours, _ = t5_pair
    for s in STRINGS + [f"Answer the organ question: {x}" for x in STRINGS[:200]]:
        assert ours._sp_encode(s) == ours.sp.EncodeAsIds(s), s


def test_t5_truncation_and_eos(t5_pair):
    ours, hf = t5_pair
    long = " ".join(["liver"] * 700)
    a = ours([long, "lung"], padding="longest", max_length=512, truncation=True)
    b = hf([long, "lung"], padding="longest", max_length=512, truncation=True)
    assert _rows(a) == _rows(b)
    assert len(a["input_ids"][0]) == 512 and a["input_ids"][0][-1] == 1
    # 4.26.1's _add_eos_if_not_present: a literal trailing </s> is the EOS
    r = ours("the answer </s>")["input_ids"]
    assert r[-1] == 1 and r[-2] != 1
    assert ours("")["input_ids"] == [1]


def test_t5_decode_matches_transformers(t5_pair):
    ours, hf = t5_pair
    rng = np.random.Generator(np.random.PCG64(5))
    seqs = []
    for s in STRINGS[:400]:
        seqs.append(ours(s)["input_ids"])
    # random id runs (greedy outputs of untrained weights look like this), with pads/eos
    for _ in range(200):
        n = int(rng.integers(1, 21))
        seqs.append([0] + rng.integers(3, 32000, size=n).tolist() + [1, 0, 0])
    for s in seqs:
        a = ours.decode(s, skip_special_tokens=True)
        b = hf.decode(s, skip_special_tokens=True, clean_up_tokenization_spaces=True)
        # 4.26.1's convert_tokens_to_string strips the decoded string; 5.x does not
        assert a == b.strip(), (s, a, b)
    assert ours.batch_decode(torch.tensor([[0, 3, 30, 1, 0]]), skip_special_tokens=True) == \
        [hf.decode([0, 3, 30, 1, 0], skip_special_tokens=True,
                   clean_up_tokenization_spaces=True).strip()]
    # the added token decodes as itself, space-joined (4.26.1 _decode)
    assert ours.decode([3, 32100, 30, 1], skip_special_tokens=True) == "the [itk] organ"


def test_t5_batch_decode_equals_per_row_decode():
    """batch_decode's batched SentencePiece path (rows without added tokens) gives decode()'s
    string for every row: random greedy-like ids with pads, eos, extra ids and the added [itk]."""
    tok = tk.SpmT5Tokenizer()
    tok.add_tokens(["[itk]"])
    g = torch.Generator().manual_seed(3)
    ids = torch.randint(3, 32000, (300, 21), generator=g)
    ids[:7, 4] = 32100          # the added token: the per-row path
    ids[7:20, 0] = 0            # pads and eos runs
    ids[20:40, 9:] = 1
    ids[40:50, 2] = 32050       # an extra id (special)
    want = [tok.decode(r.tolist(), skip_special_tokens=True) for r in ids]
    for seq in (ids, ids.to(torch.int32), ids.numpy()):
        assert tok.batch_decode(seq, skip_special_tokens=True) == want
    assert tok.batch_decode(ids, skip_special_tokens=False) == \
        [tok.decode(r.tolist()) for r in ids]
    # the per-id tables follow tokens added after a first batch decode (the new id takes the
    # per-row path; unknown ids are special and dropped as decode() drops them)
    tok.add_tokens(["[new]"])
    new_id = max(tok.added_tokens_decoder)
    ids[50:60, 5] = new_id
    ids[60:70, 6] = 2
    want = [tok.decode(r.tolist(), skip_special_tokens=True) for r in ids]
    assert tok.batch_decode(ids, skip_special_tokens=True) == want
    assert any("[new]" in w for w in want)
