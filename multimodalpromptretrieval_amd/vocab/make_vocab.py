"""Generate the stand-in tokenizer vocabularies (run once, in the build container; outputs
committed next to this file).

The reference tokenizes with openai CLIP's byte-level BPE (``clip.tokenize``,
dataset/VQAFeatureDataset.py:190; vocab ``bpe_simple_vocab_16e6.txt.gz``) and T5's SentencePiece
unigram model (``T5Tokenizer.from_pretrained("t5-small")``, architectures/T5VisionModel.py:57).
Neither vocabulary exists offline, so the tokenizers in ``tokenizers.py`` run
on vocabularies of the same FORMAT and size, learned here from English text available in this
container (comments and docstrings of the Python standard library and a few installed packages,
plus medical-VQA-style template sentences):

* ``clip_bpe_synthetic.txt.gz`` — openai-CLIP merges file: a ``#version`` header line, then
  49152 - 256 - 2 = 48,894 merges in rank order, so the vocabulary is 256 byte symbols + their
  ``</w>`` forms + the merges + ``<|startoftext|>`` (49406) + ``<|endoftext|>`` (49407), exactly
  the real vocabulary's layout.  Merges are learned with the tokenizers library's BPE trainer
  under CLIP's pre-split (its regex, lower-casing, byte-level symbols, ``</w>`` word ends).
* ``t5_spiece_synthetic.model`` — a SentencePiece unigram model of 32,000 pieces with T5's
  special ids (pad 0, eos 1, unk 2, no bos), so ``[itk]`` lands on 32,100 after the 100
  ``<extra_id_*>`` sentinels as in the reference (architectures/T5VisionModel.py:57-60).

Usage: python -m multimodalpromptretrieval_amd.vocab.make_vocab  (a few minutes, 8 threads)
"""
from __future__ import annotations

import glob
import gzip
import io
import os
import tokenize

HERE = os.path.dirname(os.path.abspath(__file__))
CLIP_MERGES = 49152 - 256 - 2
T5_PIECES = 32000
SOURCES = ["/usr/lib/python3.10",
           "/usr/local/lib/python3.10/dist-packages/transformers",
           "/usr/local/lib/python3.10/dist-packages/sklearn",
           "/usr/local/lib/python3.10/dist-packages/pandas"]

ORGANS = ("lung liver brain heart kidney spleen pancreas bladder colon rectum stomach esophagus "
          "trachea aorta spine rib femur pelvis skull uterus prostate gallbladder duodenum "
          "thyroid adrenal").split()
MODALITIES = "CT MRI X-Ray ultrasound PET T1 T2 FLAIR DWI angiography".split()
ABNORMAL = ("nodule mass effusion pneumothorax cardiomegaly edema infiltration atelectasis "
            "consolidation fracture tumor cyst hemorrhage infarct stone lesion").split()
TEMPLATES = [
    "What is the organ shown in this image?", "Which organ is abnormal?",
    "Does the picture contain {o}?", "Is the {o} healthy?", "What modality is used to take this "
    "image?", "Is this a {m} scan?", "Where is the {a} located?", "What is the largest organ in "
    "the picture?", "Which part of the body does this image belong to?", "Is there {a} in the "
    "{o}?", "What diseases are included in the picture?", "How many {o}s are there?",
    "In which plane is this image taken?", "Is the {a} on the left or right side?",
    "What color is the {o} in the image?", "Does the {o} look normal?",
    "Which is bigger in this image, the {o} or the {o2}?", "Answer the {t} question: ",
    "I believe the answer is {q} {o}", "The most frequent answer is {a}"]
TASKS = ["organ", "modality", "position", "abnormality", "plane", "quantity", "color", "size"]
QUANT = ["very unlikely", "unlikely", "maybe", "likely", "very likely", "certainly"]


def _vqa_sentences(n: int):
    import numpy as np
    rng = np.random.Generator(np.random.PCG64(88))
    for _ in range(n):
        t = TEMPLATES[int(rng.integers(len(TEMPLATES)))]
        yield t.format(o=ORGANS[int(rng.integers(len(ORGANS)))],
                       o2=ORGANS[int(rng.integers(len(ORGANS)))],
                       m=MODALITIES[int(rng.integers(len(MODALITIES)))],
                       a=ABNORMAL[int(rng.integers(len(ABNORMAL)))],
                       t=TASKS[int(rng.integers(len(TASKS)))],
                       q=QUANT[int(rng.integers(len(QUANT)))])


def _text_of(path: str):
    """Comment and string-literal text of one Python file (natural language, mostly)."""
    try:
        with open(path, "rb") as f:
            toks = list(tokenize.tokenize(io.BytesIO(f.read()).readline))
    except (tokenize.TokenError, SyntaxError, UnicodeDecodeError, IndentationError):
        return
    for t in toks:
        if t.type == tokenize.COMMENT:
            s = t.string.lstrip("#").strip()
        elif t.type == tokenize.STRING:
            s = t.string.strip("\"'rbfuRBFU")
        else:
            continue
        for line in s.splitlines():
            line = line.strip()
            letters = sum(c.isalpha() for c in line)
            if len(line) >= 12 and letters >= 0.6 * len(line):
                yield line


def corpus_lines():
    for root in SOURCES:
        for p in sorted(glob.glob(os.path.join(root, "**", "*.py"), recursive=True)):
            yield from _text_of(p)
    yield from _vqa_sentences(200_000)


def write_corpus(path: str) -> int:
    n = 0
    with open(path, "w", encoding="utf-8") as f:
        for line in corpus_lines():
            f.write(line + "\n")
            n += 1
    return n


def train_clip_bpe(corpus: str, out_gz: str) -> int:
    from tokenizers import Regex, Tokenizer, normalizers, pre_tokenizers
    from tokenizers.models import BPE
    from tokenizers.trainers import BpeTrainer
    tok = Tokenizer(BPE(end_of_word_suffix="</w>", continuing_subword_prefix=""))
    tok.normalizer = normalizers.Sequence(
        [normalizers.NFC(), normalizers.Replace(Regex(r"\s+"), " "), normalizers.Lowercase()])
    tok.pre_tokenizer = pre_tokenizers.Sequence([
        pre_tokenizers.Split(Regex(r"""<\|startoftext\|>|<\|endoftext\|>|'s|'t|'re|'ve|'m|'ll|'d|"""
                                   r"""[\p{L}]+|[\p{N}]|[^\s\p{L}\p{N}]+"""),
                             behavior="removed", invert=True),
        pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False)])
    alphabet = pre_tokenizers.ByteLevel.alphabet()
    trainer = BpeTrainer(vocab_size=2 * 256 + CLIP_MERGES + 2 + 4096, min_frequency=1,
                         initial_alphabet=alphabet, end_of_word_suffix="</w>",
                         show_progress=False, special_tokens=[])
    tok.train([corpus], trainer)
    import json
    model = json.loads(tok.to_str())["model"]
    merges = model["merges"][:CLIP_MERGES]
    with gzip.GzipFile(out_gz, "wb", mtime=0) as f:
        f.write(b"#version: 0.2 - synthetic stand-in (multimodalpromptretrieval_amd/vocab)\n")
        for m in merges:
            a, b = m if isinstance(m, (list, tuple)) else m.split(" ")
            f.write(f"{a} {b}\n".encode("utf-8"))
    return len(merges)


def train_t5_spm(corpus: str, prefix: str) -> None:
    import sentencepiece as spm
    spm.SentencePieceTrainer.train(
        input=corpus, model_prefix=prefix, vocab_size=T5_PIECES, model_type="unigram",
        pad_id=0, eos_id=1, unk_id=2, bos_id=-1, pad_piece="<pad>", eos_piece="</s>",
        unk_piece="<unk>", character_coverage=0.9995, num_threads=8,
        input_sentence_size=3_000_000, shuffle_input_sentence=False,
        normalization_rule_name="nmt_nfkc", minloglevel=2)


def main():
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        corpus = os.path.join(d, "corpus.txt")
        n = write_corpus(corpus)
        print(f"corpus: {n} lines, {os.path.getsize(corpus) / 1e6:.1f} MB")
        m = train_clip_bpe(corpus, os.path.join(HERE, "clip_bpe_synthetic.txt.gz"))
        print(f"clip: {m} merges")
        train_t5_spm(corpus, os.path.join(d, "t5"))
        os.replace(os.path.join(d, "t5.model"), os.path.join(HERE, "t5_spiece_synthetic.model"))
        print("t5: spiece written")


if __name__ == "__main__":
    main()
